set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_stamps.py > gpurun_out/gemm_stamps_r1q.log 2>&1
echo "exit=$?"
