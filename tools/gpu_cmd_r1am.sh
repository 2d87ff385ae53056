set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r1am.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r1am.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r1am.log
timeout -k 10 300 python -u tools/attn_ks_tune.py > gpurun_out/attn_ks_r1am.log 2>&1
echo "exit=$?"
