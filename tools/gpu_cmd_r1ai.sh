set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vit.py -x -v -s -k "fp8" --timeout 300 --timeout-method thread > gpurun_out/pytest_fp8_r1ai.log 2>&1
echo "exit=$?"
