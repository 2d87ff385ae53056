"""In-block key-split sweep of the attention kernel (M3S_ATTN_AW / M3S_ATTN_KS) on the
encoder / decoder / mono-decoder shapes at S = 768 and 1024.  Usage: python tools/attn_ks_tune.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd"), os.path.join(ROOT, "tools")]
from fp8_tune import graph_us, ops  # noqa: E402

dev = torch.device("cuda:0")
for S in (768, 1024):
    for name, b, heads in [("enc", 1, 16), ("dec x4", 4, 12), ("mono x2", 2, 12), ("graph x32", 32, 12)]:
        C = heads * 64
        qkv = torch.randn(b, S, 3 * C, device=dev).bfloat16()
        o = torch.empty(b, S, C, device=dev, dtype=torch.bfloat16)
        fl = 4.0 * S * S * 64 * heads * b
        line = f"S{S} {name:10s}"
        for aw, ks in [("4", "1"), ("2", "1"), ("4", "2"), ("2", "2"), ("2", "4")]:
            os.environ["M3S_ATTN_AW"], os.environ["M3S_ATTN_KS"] = aw, ks
            us = graph_us(lambda: ops.attn(qkv, 3 * C, S * 3 * C, qkv[:, :, C:], qkv[:, :, 2 * C:],
                                           3 * C, S * 3 * C, o, C, S * C, b, heads, S, S))
            line += f" aw{aw}ks{ks} {us:6.1f}us {fl / us / 1e6:4.0f}TF"
        print(line, flush=True)
