set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pr in "0 0" "-1 0" "0 -1" "-1 1" ; do
  set -- $pr
  timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --no-graph --no-c5 --main-priority $1 --side-priority $2 > gpurun_out/bench_r1ap_$1_$2.json 2>gpurun_out/bench_r1ap.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_r1ap_$1_$2.json').read().strip().splitlines()[-1]); print('main $1 side $2', d['value'])"
done
echo "exit=$?"
