set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu_r1l.log 2>&1; echo "pytest rc=$?"
timeout -k 10 700 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1l.log 2>&1; echo "tune rc=$?"
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1l.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_l -o bench --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace_r1l.log 2>&1
echo "exit=$?"
