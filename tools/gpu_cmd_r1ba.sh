# Re-entry validation of HEAD: GPU tests, smoke, default bench (with cpu_baseline),
# kernel-trace stats, per-shape GEMM breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_ba
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1ba.log 2>&1 && tail -1 gpurun_out/pytest_gpu_r1ba.log && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r1ba.log 2>&1 && tail -1 gpurun_out/smoke_r1ba.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1ba.json 2> gpurun_out/bench_r1ba.err && cat gpurun_out/bench_r1ba.json && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ba/trace -o bench --output-format csv \
    -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_ba/bench_traced.json 2> gpurun_out/prof_ba/trace.log && \
timeout -k 10 200 python -u tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_r1ba.log 2>&1
echo "exit=$?"
