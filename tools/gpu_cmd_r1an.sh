set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1an.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r1an.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r1an.log
timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-graph > gpurun_out/bench_r1an.json 2> gpurun_out/bench_r1an.err
echo "bench exit=$?"
