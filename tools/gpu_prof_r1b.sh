# Profiling pass: kernel-trace stats of the default bench command, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) on the pair probe.  Each step has its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv \
    -- python3 bench.py > gpurun_out/prof/bench_traced.json 2> gpurun_out/prof/trace.log && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/pmc_hit -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/hit.log 2>&1
echo "exit=$?"
