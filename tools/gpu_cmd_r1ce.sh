# validation: all GPU tests (incl. retrieval + harness), smoke, default bench, kernel-trace stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 200 python -u -m pytest tests/test_gpu_harness.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_harness_r1ce.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_harness_r1ce.log
[ $rc -eq 0 ] || { echo "harness test failed rc=$rc"; grep -n "Error\|assert\|rmse" gpurun_out/pytest_harness_r1ce.log | head -30; exit 1; }
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1ce.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r1ce.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_r1ce.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1ce.log 2>&1 || { tail -30 gpurun_out/smoke_r1ce.log; exit 1; }
tail -1 gpurun_out/smoke_r1ce.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1ce.json 2> gpurun_out/bench_r1ce.err || { tail -30 gpurun_out/bench_r1ce.err; exit 1; }
cat gpurun_out/bench_r1ce.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r1ce -o r1ce --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench_prof_r1ce.log 2>&1 || { tail -30 gpurun_out/bench_prof_r1ce.log; exit 1; }
echo "exit=$?"
