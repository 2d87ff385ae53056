set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof4/blas -o blas --output-format csv -- python3 tools/blas_probe.py > gpurun_out/blas_probe.log 2>&1
echo "exit=$?"
