set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fp8_tune.py > gpurun_out/fp8_tune_r1ak.log 2>&1
echo "exit=$?"
