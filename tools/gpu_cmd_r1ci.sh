# tracker GN: vectorised partial-row reduction — tracker/sequence GPU tests, bench x2, kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_gn_tracker.py tests/test_gpu_sequence.py tests/test_gpu_harness.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_trk_r1ci.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_trk_r1ci.log
[ $rc -eq 0 ] || { echo "tracker tests failed rc=$rc"; tail -40 gpurun_out/pytest_trk_r1ci.log; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --no-retrieval --steps 200 > gpurun_out/bench_a${i}_r1ci.json 2> gpurun_out/bench_a${i}_r1ci.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1ci.json'));print('fps', d['value'], d['tracker_gn'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r1ci -o r1ci --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-graph --no-c5 --no-retrieval > gpurun_out/bench_prof_r1ci.log 2>&1 || { tail -30 gpurun_out/bench_prof_r1ci.log; exit 1; }
grep -E "track_" gpurun_out/prof/r1ci/r1ci_kernel_stats.csv | cut -c1-200
