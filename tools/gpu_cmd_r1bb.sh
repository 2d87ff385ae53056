# DMA-ring depth sweep on the M = 768 shapes + per-phase stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_depth.py > gpurun_out/gemm_depth_r1bb.log 2>&1 && cat gpurun_out/gemm_depth_r1bb.log && \
timeout -k 10 200 python -u tools/gemm_stamps.py > gpurun_out/gemm_stamps_r1bb.log 2>&1 && cat gpurun_out/gemm_stamps_r1bb.log
echo "exit=$?"
