# A/B of the tile rules on long benches (200 steps each, alternating).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_a${i}_r1bk.json 2> gpurun_out/bench_a${i}_r1bk.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1bk.json'));print('new', d['value'], d['roofline']['gemm_ms_per_pair'])"
M3S_NO_T96=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --steps 200 > gpurun_out/bench_b${i}_r1bk.json 2> gpurun_out/bench_b${i}_r1bk.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_b${i}_r1bk.json'));print('no96', d['value'], d['roofline']['gemm_ms_per_pair'])"
done
echo "exit=$?"
