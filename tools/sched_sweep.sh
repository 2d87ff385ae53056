# Pipelined C3 step time per setting: one bench run (no timeline / extra legs) per spec.
# A spec is space-separated VAR=value environment assignments and/or bench.py flags, e.g.
#   bash tools/sched_sweep.sh "" "M3S_ENC_TILE=qkv=13:1,proj=14:1,fc1=14:1,fc2=14:1" "--group 1"
# Prints "<spec> <frames/s> <ms/step>" per line; stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  envs=(); flags=()
  for w in $spec; do
    if [[ "$w" == --* || ${#flags[@]} -gt 0 ]]; then flags+=("$w"); else envs+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-graph --no-c5 --no-retrieval \
      --no-cpu-baseline --no-timeline --steps 200 "${flags[@]}" \
      > gpurun_out/sched_sweep.json 2> gpurun_out/sched_sweep.err || { tail -20 gpurun_out/sched_sweep.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sched_sweep.json').read().strip().splitlines()[-1]);print(repr('$spec'), round(d['value'],1), 'fps', round(d['ms_per_step'],3), 'ms', 'pair', round(d['pair_inference_ms'] or 0,3), 'ms')"
done
