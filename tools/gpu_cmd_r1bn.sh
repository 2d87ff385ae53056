# fused glue + refinenet skip-in-upsample + lf side: GPU tests, A/B fused glue.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1bn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r1bn.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_r1bn.log; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_a${i}_r1bn.json 2> gpurun_out/bench_a${i}_r1bn.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1bn.json'));print('fused', d['value'], d['tracker_gn'])"
M3S_FUSED_GLUE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_b${i}_r1bn.json 2> gpurun_out/bench_b${i}_r1bn.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_b${i}_r1bn.json'));print('torch', d['value'], d['tracker_gn'])"
done
echo "exit=$?"
