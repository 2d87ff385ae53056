set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/trace -o bench --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-graph > gpurun_out/prof_trace_r1ac.log 2>&1
echo "exit=$?"
