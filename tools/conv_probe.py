"""The pair's largest DPT convs replayed alone (tools only): records one pair inference's
GEMM launches (bench.gemm_replay's descriptors), keeps the implicit-conv launches with
M >= 12288, and times each shape replayed back to back in a HIP graph; under
`rocprofv3 --pmc FETCH_SIZE` the per-dispatch bytes show how often the conv's input
is re-read beyond L2.  Prints one line per shape: us per launch, TF/s, algorithmic bytes
(input image once + weights + output), marker-bracketed for the PMC parser.
  python tools/conv_probe.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    model, tr, seq = bench.setup(dev, 0, 4)
    img = seq.img[1]
    feat_k, _ = model.encode(seq.img[0])
    feat_k = feat_k.clone()
    model.serial, model.dec_split = True, False
    ops = model.ops
    ops.record = []
    model.pair(img, feat_j=feat_k)
    torch.cuda.synchronize(dev)
    rec, ops.record = ops.record, None
    convs = {}
    for d, fl, f8 in rec:
        if d.mode != 0 and d.M >= 12288:
            convs.setdefault((d.M, d.N, d.K, d.batch, d.flags), (d, fl))
    for key, (d, fl) in sorted(convs.items(), key=lambda kv: -kv[1][1]):
        g = bench.capture(lambda d=d: [ops.replay_gemm(d) for _ in range(reps)], dev)
        ms = bench.time_replays(g, dev, 5) / reps
        M, N, K, b, flags = key
        cin = K // 9
        # input image once (stride 1) + weights + output (the fused DPT tail writes 16 B
        # per pixel instead of the 128-channel map)
        out_b = M * 16 if flags & 512 else M * N * 2
        alg = (M * cin * 2 + out_b) * b + N * K * 2
        print(f"conv M={M} N={N} K={K} b={b} flags={flags}: {ms * 1e3:.1f} us, "
              f"{fl / ms / 1e9:.0f} TF/s, algorithmic {alg / 1e6:.1f} MB "
              f"({alg / ms / 1e6:.0f} GB/s)", flush=True)
        del g


if __name__ == "__main__":
    main()
