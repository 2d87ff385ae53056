set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vit.py -q -rf -s > gpurun_out/pytest_vit_r1d.log 2>&1 || { echo "pytest failed $?"; }
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench_v3.log 2>&1 && \
timeout -k 10 300 python tools/gemm_breakdown.py > gpurun_out/gemm_breakdown_v3.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1d.log 2>&1; echo "exit=$?"
