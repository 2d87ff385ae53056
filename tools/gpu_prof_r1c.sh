# Full GPU tests, default bench, kernel-trace stats of the default bench, PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1c.log 2>&1 && tail -1 gpurun_out/pytest_gpu_r1c.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1c.json 2> gpurun_out/bench_r1c.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv \
    -- python3 bench.py > gpurun_out/prof/bench_traced.json 2> gpurun_out/prof/trace.log && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/pmc_hit -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-graph > gpurun_out/prof/hit.log 2>&1
echo "exit=$?"
