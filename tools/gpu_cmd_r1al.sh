set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c5_prof.py 20 > gpurun_out/c5_r1al.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 tools/c5_prof.py 5 > gpurun_out/c5_prof_r1al.log 2>&1
echo "exit=$?"
