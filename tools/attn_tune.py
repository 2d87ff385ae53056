"""Attention timing (graph-replayed) over waves-per-block and key splits, encoder
(1 x 16 heads) and decoder (4 x 12 heads) shapes, 768 tokens, head dim 64."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")


def graph_us(fn, rep=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(rep):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / rep)
    return best

ops = Ops(dev)
for name, b, heads in [("attn enc", 1, 16), ("attn dec x4", 4, 12)]:
    S, C = 768, heads * 64
    qkv = torch.randn(b, S, 3 * C, device=dev).bfloat16()
    o = torch.empty(b, S, C, device=dev, dtype=torch.bfloat16)
    fl = 4.0 * S * S * 64 * heads * b
    line = f"{name:12s}"
    for aw in ("2", "4"):
        for sp in ("", "2", "4"):
            os.environ["M3S_ATTN_AW"] = aw
            os.environ.pop("M3S_ATTN_SPLITS", None)
            os.environ.pop("M3S_ATTN_NOPIPE", None)
            if sp == "nopipe":
                os.environ["M3S_ATTN_NOPIPE"] = "1"
            elif sp:
                os.environ["M3S_ATTN_SPLITS"] = sp
            us = graph_us(lambda: ops.attn(qkv, 3 * C, S * 3 * C, qkv[:, :, C:], qkv[:, :, 2 * C:],
                                           3 * C, S * 3 * C, o, C, S * C, b, heads, S, S))
            line += f" aw{aw}s{sp or 'auto'} {us:5.1f}"
    os.environ.pop("M3S_ATTN_AW", None)
    os.environ.pop("M3S_ATTN_SPLITS", None)
    os.environ.pop("M3S_ATTN_NOPIPE", None)
    us = graph_us(lambda: ops.attn(qkv, 3 * C, S * 3 * C, qkv[:, :, C:], qkv[:, :, 2 * C:],
                                   3 * C, S * 3 * C, o, C, S * C, b, heads, S, S))
    print(line + f" | default {us:.1f}us {fl / us / 1e6:.0f}TF", flush=True)
