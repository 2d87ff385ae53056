#!/bin/bash
# Round-end GPU checks (run from the repo root on the GPU box): the whole -m gpu suite,
# then smoke(); each under its own time limit, the first failure ends the script.
#   bash tools/gpu_suite.sh [R]   → gpurun_out/${R}_gpu_tests.txt, gpurun_out/${R}_smoke.txt
set -o pipefail
export TMPDIR=/tmp
R=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ \
  > gpurun_out/${R}_gpu_tests.txt 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" gpurun_out/${R}_gpu_tests.txt | head -20; tail -20 gpurun_out/${R}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${R}_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/${R}_smoke.txt 2>&1; st=$?; tail -3 gpurun_out/${R}_smoke.txt; exit $st
