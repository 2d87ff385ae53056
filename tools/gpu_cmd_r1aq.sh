set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py tests/test_gpu_sequence.py -x -q -k "split or pipeline or sequence" --timeout 200 --timeout-method thread > gpurun_out/pytest_r1aq.log 2>&1 || { tail -30 gpurun_out/pytest_r1aq.log; exit 1; }
tail -1 gpurun_out/pytest_r1aq.log
timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 > gpurun_out/bench_r1aq_split.json 2>gpurun_out/bench_r1aq.err || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 --no-split-heads > gpurun_out/bench_r1aq_nosplit.json 2>>gpurun_out/bench_r1aq.err || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 --no-prefetch > gpurun_out/bench_r1aq_split_noprefetch.json 2>>gpurun_out/bench_r1aq.err
for f in split nosplit split_noprefetch; do python -c "import json; d=json.loads(open('gpurun_out/bench_r1aq_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['pair_inference_ms'])"; done
echo "exit=$?"
