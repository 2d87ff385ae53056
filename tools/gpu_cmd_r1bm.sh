# A/B: local features on the side chain (split heads) vs on the tracking chain.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sequence.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_seq_r1bm.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_seq_r1bm.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_a${i}_r1bm.json 2> gpurun_out/bench_a${i}_r1bm.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1bm.json'));print('lf_side', d['value'])"
M3S_LF_SIDE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_b${i}_r1bm.json 2> gpurun_out/bench_b${i}_r1bm.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_b${i}_r1bm.json'));print('lf_main', d['value'])"
done
echo "exit=$?"
