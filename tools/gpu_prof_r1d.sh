# Round profiles of the current state: default bench (with cpu_baseline), kernel-trace stats,
# PMC passes (separate runs) for the GEMM traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_d
timeout -k 10 400 python -u bench.py > gpurun_out/prof_d/bench.json 2> gpurun_out/prof_d/bench.err && cat gpurun_out/prof_d/bench.json && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d/trace -o bench --output-format csv \
    -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_d/bench_traced.json 2> gpurun_out/prof_d/trace.log && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_d/pmc_fetch -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof_d/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_d/pmc_write -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof_d/write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_d/pmc_hit -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof_d/hit.log 2>&1
echo "exit=$?"
