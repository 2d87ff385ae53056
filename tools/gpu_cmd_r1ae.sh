set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-graph > gpurun_out/bench_r1ae_at$i.log 2>&1 && \
M3S_GEMM_NO_ATOMIC=1 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-graph > gpurun_out/bench_r1ae_na$i.log 2>&1 || exit 1
done
echo "exit=$?"
