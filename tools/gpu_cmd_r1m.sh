# Re-entry check: GPU parity tests, smoke, full bench (with cpu_baseline), kernel-trace stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1m.log 2>&1 && \
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r1m.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_r1m.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_m -o bench --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace_r1m.log 2>&1
echo "exit=$?"
