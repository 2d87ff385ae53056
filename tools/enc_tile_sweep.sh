# Pipelined C3 step time per encoder tile configuration (PairModel.encode(concurrent=True),
# M3S_ENC_TILE knob): one bench run per setting, on the GPU box via gpurun.
#   bash tools/enc_tile_sweep.sh "table" "12:1" "qkv=12:1,proj=1:1,fc1=12:1,fc2=12:1" ...
# KNOB=M3S_DEC_TILE sweeps the decoder's projections (qkv, proj, q, cproj, fc1, fc2) instead,
# KNOB=M3S_SIDE_TILE the split-heads side chain (lf = local-feature MLP, dpt = MASt3R heads).
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  export ${KNOB:-M3S_ENC_TILE}="$v"
  timeout -k 10 240 python -u bench.py --no-graph --no-c5 --no-retrieval --no-cpu-baseline --steps 200 \
      > gpurun_out/enc_sweep.json 2> gpurun_out/enc_sweep.err || { tail -20 gpurun_out/enc_sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/enc_sweep.json'));print('$v', round(d['value'],1), 'fps', round(d['ms_per_step'],3), 'ms')"
done
