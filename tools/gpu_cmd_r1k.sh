set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vit.py -x -q -rf > gpurun_out/pytest_vit_r1k.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python tools/gemm_stamps.py > gpurun_out/stamps5.log 2>&1; echo "stamps rc=$?"
timeout -k 10 700 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1k.log 2>&1; echo "tune rc=$?"
