# retrieval kernels: GPU parity tests, bench retrieval leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_retr_r1cg.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_retr_r1cg.log
[ $rc -eq 0 ] || { echo "retrieval tests failed rc=$rc"; grep -n "Error\|assert" gpurun_out/pytest_retr_r1cg.log | head -40; exit 1; }
timeout -k 10 300 python -u bench.py --no-graph --no-c5 --steps 10 > gpurun_out/bench_r1cg.json 2> gpurun_out/bench_r1cg.err || { tail -30 gpurun_out/bench_r1cg.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r1cg.json'));print(d['value']);print(json.dumps(d['keyframe_retrieval'],indent=1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r1cg -o r1cg --output-format csv -- python3 bench.py --steps 4 --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_prof_r1cg.log 2>&1 || { tail -30 gpurun_out/bench_prof_r1cg.log; exit 1; }
grep -E "quantize|affine|aggregate|ivf_score|topk|rownorm|words" gpurun_out/prof/r1cg/r1cg_kernel_stats.csv | cut -c1-150
