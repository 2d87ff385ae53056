# PMC passes over a short bench run (one counter group per pass, as the guide prescribes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/pmc_hit -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/pmc_hit.log 2>&1
echo "exit=$?"
