# GPU: full gpu test suite (incl. new keyframe-graph / dynamic-mask tests).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1o.log 2>&1
echo "exit=$?"
