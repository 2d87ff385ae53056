# Full GPU tests + default bench (with cpu_baseline) + 200-step headline A/B repeat.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1bl.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r1bl.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_r1bl.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1bl.json 2> gpurun_out/bench_r1bl.err && cat gpurun_out/bench_r1bl.json || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_a${i}_r1bl.json 2> gpurun_out/bench_a${i}_r1bl.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1bl.json'));print('default', d['value'], d['roofline']['gemm_ms_per_pair'])"
done
echo "exit=$?"
