set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1ad.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r1ad.log 2>&1 && \
timeout -k 10 700 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1ad.log 2>&1
echo "exit=$?"
