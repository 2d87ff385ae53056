#!/bin/bash
# Round-end GPU evidence for the bench line (run from the repo root on the GPU box):
#   bash tools/gpu_final.sh bench    the default bench line (all legs) → gpurun_out/$R_bench.json
#   bash tools/gpu_final.sh prof     rocprofv3 kernel trace + MFMA PMC pass of the timed C3 step
#                                    (tools/step_prof.py) → gpurun_out/$R_step_pmc.json
# Each GPU step runs under its own time limit; a failing step ends the script.
set -o pipefail
export TMPDIR=/tmp
R=${R:-r03}
mkdir -p gpurun_out
case "$1" in
  bench)
    timeout -k 10 600 python -u bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err \
      || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
    tail -c 400 gpurun_out/${R}_bench.json ;;
  prof)
    ms=$(python -c "import json;print(json.loads(open('gpurun_out/${R}_bench.json').read().strip().splitlines()[-1])['ms_per_step'])" 2>/dev/null || echo 4.3)
    rm -rf gpurun_out/${R}_trace gpurun_out/${R}_pmc
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o step -- \
      python3 tools/step_prof.py --steps 20 > gpurun_out/${R}_trace.log 2>&1 \
      || { tail -20 gpurun_out/${R}_trace.log; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU GRBM_GUI_ACTIVE \
      --output-format csv -d gpurun_out/${R}_pmc -o step -- python3 tools/step_prof.py --steps 20 \
      > gpurun_out/${R}_pmc.log 2>&1 || { tail -20 gpurun_out/${R}_pmc.log; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
      rm -rf gpurun_out/${R}_pmc_$c
      timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${R}_pmc_$c -o step -- \
        python3 tools/step_prof.py --steps 20 > gpurun_out/${R}_pmc_$c.log 2>&1 \
        || { tail -20 gpurun_out/${R}_pmc_$c.log; exit 1; }
    done
    python tools/step_pmc_report.py --pmc gpurun_out/${R}_pmc --trace gpurun_out/${R}_trace \
      --fetch gpurun_out/${R}_pmc_FETCH_SIZE --write gpurun_out/${R}_pmc_WRITE_SIZE \
      --steps 20 --step-ms "$ms" --out gpurun_out/${R}_step_pmc.json || exit 1
    # keep the summaries, drop the raw traces (gpurun copies back at most 64 MiB)
    f=$(find gpurun_out/${R}_trace -name "*kernel_stats.csv" | head -1)
    [ -n "$f" ] && cp "$f" gpurun_out/${R}_step_kernel_stats.csv
    rm -rf gpurun_out/${R}_trace gpurun_out/${R}_pmc gpurun_out/${R}_pmc_FETCH_SIZE \
      gpurun_out/${R}_pmc_WRITE_SIZE
    tail -c 600 gpurun_out/${R}_step_pmc.json ;;
  *) echo "usage: $0 bench|prof"; exit 2 ;;
esac
