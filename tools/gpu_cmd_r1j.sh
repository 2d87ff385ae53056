set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 python tools/match_bench.py > gpurun_out/match_bench_r1j.log 2>&1; echo "mb rc=$?"
timeout -k 10 300 python tools/gemm_stamps.py > gpurun_out/stamps4.log 2>&1; echo "stamps rc=$?"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu_r1j.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1j.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_j -o bench --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace_r1j.log 2>&1
echo "exit=$?"
