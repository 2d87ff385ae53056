"""What a frame-pair batched pair inference would cost (C3 schedule question, round 6):
graph-replayed decode_multi + heads for G = 1 directed pair (the C3 step's one frame:
split decoder chains, split heads) against G = 2 (two frames vs the same keyframe in one
batch: Z = 8 problems per launch) — per-frame cost ratio.  HIP events around graph replays.
Usage: python tools/pair_batch_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
H, W = 384, 512
gh, gw = H // 16, W // 16
S, E = gh * gw, m.a.enc_dim
g = torch.Generator(device=dev).manual_seed(0)
img = torch.rand(3, 3, H, W, device=dev, generator=g) * 2 - 1
feats = torch.stack([m.encode(img[i:i + 1])[0][0].clone() for i in range(3)])  # [3,S,E]
kf = feats[2:3].contiguous()


def run(G, split, heads=True):
    f1 = feats[0:G].contiguous()
    f2 = kf.expand(G, S, E).contiguous()
    if G == 1 and split:
        hooks = m.decode(f1[0], f2[0], m.positions(1, gh, gw), gh, gw)
        if heads:
            m.heads(hooks, gh, gw, H, W, split=True)
            m.join()
    else:
        hooks = m.decode_multi(f1, f2, gh, gw)
        if heads:
            m.heads(hooks, gh, gw, H, W)


res = {}
for name, G, split, heads in (("G1 split dec", 1, True, False), ("G1 split dec+heads", 1, True, True),
                              ("G1 one-chain dec", 1, False, False),
                              ("G1 one-chain dec+heads", 1, False, True),
                              ("G2 one-chain dec", 2, False, False),
                              ("G2 one-chain dec+heads", 2, False, True)):
    for _ in range(2):
        run(G, split, heads)
    torch.cuda.synchronize()
    gr = bench.capture(lambda: run(G, split, heads), dev)
    ms = min(bench.time_replays(gr, dev, 20) for _ in range(3))
    del gr
    res[name] = ms
    print(f"{name:26s} {ms:7.3f} ms  ({ms / G:7.3f} ms per frame)", flush=True)
