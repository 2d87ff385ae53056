set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof/attnp -o attnp --output-format csv -- python3 tools/attn_probe.py > gpurun_out/attn_probe_r1w.log 2>&1
echo "exit=$?"
