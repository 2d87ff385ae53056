# Kernel-boundary cost in a replayed graph.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/launch_cost.py > gpurun_out/launch_cost_r1bc.log 2>&1; rc=$?
cat gpurun_out/launch_cost_r1bc.log
echo "exit=$rc"
