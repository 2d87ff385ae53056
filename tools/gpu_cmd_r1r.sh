set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1r.log 2>&1
echo "exit=$?"
