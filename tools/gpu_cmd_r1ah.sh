set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -v -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8_r1ah.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vit_r1ah.log 2>&1
echo "exit=$?"
