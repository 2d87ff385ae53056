"""Graph-replayed timing of the 768/1024-token attention launches, lockstep (M3S_ATTN_PP=0)
vs ping-pong (1) kernel: encoder (16 heads, batch 1, 2 x 4 waves), pair decoder (12 heads,
batch 2, 4 x 2 waves), 20 launches x 5 replays, HIP events on the replay stream."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)


def timed(fn, reps=20, replays=5):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(replays):
            g.replay()
        e1.record(s)
        e1.synchronize()
    return e0.elapsed_time(e1) / (replays * reps) * 1e3


for name, S, heads, batch in (("encoder", 768, 16, 1), ("decoder", 768, 12, 2),
                              ("enc512", 1024, 16, 1), ("dec512", 1024, 12, 2)):
    D = heads * 64
    g = torch.Generator(device=dev).manual_seed(1)
    qkv = torch.randn(batch, S, 3 * D, device=dev, generator=g).bfloat16()
    o = torch.empty(batch, S, D, device=dev, dtype=torch.bfloat16)
    fl = 4.0 * S * S * 64 * heads * batch
    res = {}
    for rnd in range(2):
        for pp in ("0", "1"):
            os.environ["M3S_ATTN_PP"] = pp
            us = timed(lambda: ops.attn(qkv, 3 * D, S * 3 * D, qkv[:, :, D:], qkv[:, :, 2 * D:],
                                        3 * D, S * 3 * D, o, D, S * D, batch, heads, S, S))
            res.setdefault(pp, []).append(us)
    print(f"{name:8s} S={S} h={heads} b={batch}: lockstep " +
          " ".join(f"{u:.1f}" for u in res["0"]) + " us | ping-pong " +
          " ".join(f"{u:.1f}" for u in res["1"]) +
          f" us ({fl / min(res['1']) / 1e6:.0f} TF/s)", flush=True)
