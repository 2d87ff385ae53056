set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gn_tracker.py tests/test_gpu_sequence.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r1ar.log 2>&1 || { tail -30 gpurun_out/pytest_r1ar.log; exit 1; }
tail -1 gpurun_out/pytest_r1ar.log
timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_r1ar_p.json 2>gpurun_out/bench_r1ar.err || exit 1
M3S_TRACK_PERSISTENT=0 timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_r1ar_np.json 2>>gpurun_out/bench_r1ar.err || exit 1
for f in p np; do python -c "import json; d=json.loads(open('gpurun_out/bench_r1ar_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['tracker_gn'])"; done
echo "exit=$?"
