# conv split-K + T128O2 head convs: GPU tests, sweep (incl. T96 on the decoder shapes), bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1bi.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_r1bi.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_r1bi.log; exit 1; }
CONVS=0 TILES=0,1,8,9,2,7 timeout -k 10 300 python -u tools/gemm_depth.py > gpurun_out/sweep_r1bi.log 2>&1; cat gpurun_out/sweep_r1bi.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_r1bi.json 2> gpurun_out/bench_r1bi.err && cat gpurun_out/bench_r1bi.json
echo "exit=$?"
timeout -k 10 300 python -u tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_r1bi.log 2>&1 && head -14 gpurun_out/gemm_breakdown_r1bi.log
