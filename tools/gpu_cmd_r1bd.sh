# Graph-replayed per-shape GEMM breakdown of one pair + tile/depth sweep.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_r1bd.log 2>&1 && cat gpurun_out/gemm_breakdown_r1bd.log && \
timeout -k 10 300 python -u tools/gemm_depth.py > gpurun_out/gemm_depth_r1bd.log 2>&1 && cat gpurun_out/gemm_depth_r1bd.log
echo "exit=$?"
