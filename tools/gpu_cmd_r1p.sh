# bench with the keyframe-graph leg (N=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1p.log 2>&1
echo "exit=$?"
