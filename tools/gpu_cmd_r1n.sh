# GEMM per-shape breakdown + tile sweep vs hipBLASLt on the pair shapes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_r1n.log 2>&1 && \
timeout -k 10 600 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1n.log 2>&1
echo "exit=$?"
