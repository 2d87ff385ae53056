# re-entry validation: GPU tests, smoke, default bench (cpu baseline + all legs), kernel-trace stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1ca.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r1ca.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_r1ca.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r1ca.log 2>&1 || { tail -30 gpurun_out/smoke_r1ca.log; exit 1; }
tail -1 gpurun_out/smoke_r1ca.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1ca.json 2> gpurun_out/bench_r1ca.err || { tail -30 gpurun_out/bench_r1ca.err; exit 1; }
cat gpurun_out/bench_r1ca.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r1ca -o r1ca --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench_prof_r1ca.log 2>&1 || { tail -30 gpurun_out/bench_prof_r1ca.log; exit 1; }
echo "exit=$?"
