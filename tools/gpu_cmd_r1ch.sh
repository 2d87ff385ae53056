# 32-bit index upsample: ViT GPU tests, bench tracking line x2, kernel stats of the tracking line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_vit_r1ch.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_vit_r1ch.log
[ $rc -eq 0 ] || { echo "vit tests failed rc=$rc"; tail -40 gpurun_out/pytest_vit_r1ch.log; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --no-c5 --no-retrieval --steps 200 > gpurun_out/bench_a${i}_r1ch.json 2> gpurun_out/bench_a${i}_r1ch.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_a${i}_r1ch.json'));print('fps', d['value'], d['pair_inference_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r1ch -o r1ch --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-graph --no-c5 --no-retrieval > gpurun_out/bench_prof_r1ch.log 2>&1 || { tail -30 gpurun_out/bench_prof_r1ch.log; exit 1; }
grep -E "upsample" gpurun_out/prof/r1ch/r1ch_kernel_stats.csv | cut -c1-200
