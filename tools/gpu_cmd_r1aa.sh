set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1aa.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r1aa.log 2>&1 && \
timeout -k 10 700 python tools/gemm_tune.py --quick > gpurun_out/gemm_tune_r1aa.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof2/pmc_fetch -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_fetch2.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof2/pmc_write -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_write2.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof2/pmc_hit -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_hit2.log 2>&1
echo "exit=$?"
