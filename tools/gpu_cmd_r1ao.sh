set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sequence.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_seq_r1ao.log 2>&1 || { tail -30 gpurun_out/pytest_seq_r1ao.log; exit 1; }
tail -1 gpurun_out/pytest_seq_r1ao.log
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_r1ao_pf.json 2> gpurun_out/bench_r1ao_pf.err || exit 1
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 --no-prefetch > gpurun_out/bench_r1ao_serial.json 2> gpurun_out/bench_r1ao_serial.err
echo "exit=$?"
