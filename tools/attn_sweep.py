"""Diagnostic: m3s_vit_attention alone (HIP graph of back-to-back launches) on the step's
shapes — decoder self / cross attention (768 tokens, 12 heads, batch 2 per split chain,
4 batched), encoder (768 tokens x 2 frames, 16 heads) — for every in-block split shape
(query waves AW x key splits KS).  Prints us per launch and TF/s.
Usage: python tools/attn_sweep.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
ops = Ops(dev)
reps = 20
g = torch.Generator(device=dev).manual_seed(1)
for name, S, heads, batch, xor in (("dec self b2", 768, 12, 2, 0), ("dec cross b2", 768, 12, 2, 1),
                                   ("dec self b4", 768, 12, 4, 0), ("enc b2", 768, 16, 2, 0),
                                   ("enc b1", 768, 16, 1, 0), ("mono512 b2", 1024, 12, 2, 0)):
    D = heads * 64
    q = torch.randn(batch, S, D, device=dev, generator=g).bfloat16()
    kv = torch.randn(batch, S, 2 * D, device=dev, generator=g).bfloat16()
    o = torch.empty(batch, S, D, device=dev, dtype=torch.bfloat16)
    fl = 4.0 * S * S * 64 * heads * batch
    row = []
    for aw, ks in (("0", "0"), ("4", "1"), ("2", "1"), ("4", "2"), ("2", "2"), ("2", "4")):
        if aw == "0":
            os.environ.pop("M3S_ATTN_AW", None)
            os.environ.pop("M3S_ATTN_KS", None)
        else:
            os.environ["M3S_ATTN_AW"], os.environ["M3S_ATTN_KS"] = aw, ks
        gr = B.capture(lambda: [ops.attn(q, D, S * D, kv, kv[:, :, D:], 2 * D, S * 2 * D, o, D,
                                         S * D, batch, heads, S, S, kv_xor=xor)
                                for _ in range(reps)], dev)
        ms = B.time_replays(gr, dev, 5) / reps
        del gr
        row.append(f"{'auto' if aw == '0' else aw + 'x' + ks}={ms * 1e3:5.1f}us/{fl / ms / 1e9:4.0f}TF")
    print(f"{name:14s} " + "  ".join(row), flush=True)
os.environ.pop("M3S_ATTN_AW", None)
os.environ.pop("M3S_ATTN_KS", None)
