set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vit.py -q -rf -s > gpurun_out/pytest_vit_r1c.log 2>&1; echo "pytest_exit=$?"
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > gpurun_out/bench_r1c.log 2>&1; echo "bench_exit=$?"
