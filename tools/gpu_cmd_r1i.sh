set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_matching.py -x -q -rf > gpurun_out/pytest_match_r1i.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python tools/match_bench.py > gpurun_out/match_bench_r1i.log 2>&1; echo "mb rc=$?"
timeout -k 10 300 python tools/gemm_stamps.py > gpurun_out/stamps3.log 2>&1; echo "stamps rc=$?"
