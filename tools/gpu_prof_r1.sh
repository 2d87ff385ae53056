# Round-1 profiling pass: full GPU tests + smoke, kernel-trace stats of bench.py, and two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic. Each step has its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu_r1.log 2>&1 && \
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/smoke_r1.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv \
    -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace_r1.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o bench --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_fetch_r1.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o bench --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_write_r1.log 2>&1
echo "exit=$?"
