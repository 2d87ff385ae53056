# LN fold + fast GELU + T64 heuristic: new tests, full GPU tests, bench, GEMM breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -m gpu -x -q -k "ln_ or gelu" --timeout 200 --timeout-method thread > gpurun_out/pytest_ln_r1be.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_ln_r1be.log
[ $rc -eq 0 ] || { echo "ln tests failed rc=$rc"; exit 1; }
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r1be.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu_r1be.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r1be.json 2> gpurun_out/bench_r1be.err && cat gpurun_out/bench_r1be.json && \
M3S_LNFOLD=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_nofold_r1be.json 2> gpurun_out/bench_nofold_r1be.err && cat gpurun_out/bench_nofold_r1be.json && \
timeout -k 10 300 python -u tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_r1be.log 2>&1 && cat gpurun_out/gemm_breakdown_r1be.log
echo "exit=$?"
