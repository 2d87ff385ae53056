# Conv tile sweep + kernel trace of the headline tracking steps only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_bg
GEMMS=0 timeout -k 10 300 python -u tools/gemm_depth.py > gpurun_out/conv_sweep_r1bg.log 2>&1; cat gpurun_out/conv_sweep_r1bg.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bg/trace -o bench --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-graph --no-c5 --steps 10 > gpurun_out/prof_bg/bench_traced.json 2> gpurun_out/prof_bg/trace.log && \
python tools/trace_streams.py gpurun_out/prof_bg/trace/bench_kernel_trace.csv > gpurun_out/prof_bg/streams.txt 2>&1; head -150 gpurun_out/prof_bg/streams.txt
echo "exit=$?"
