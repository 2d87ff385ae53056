set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/attn -o attn --output-format csv -- python3 tools/attn_tune.py > gpurun_out/attn_prof_r1v.log 2>&1
echo "exit=$?"
