set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1aj.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r1aj.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r1aj.log
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-graph > gpurun_out/bench_r1aj.json 2> gpurun_out/bench_r1aj.err
echo "bench exit=$?"
