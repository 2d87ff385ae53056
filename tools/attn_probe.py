"""Attention kernel duration vs shape (fixed-cost probe): run under rocprofv3 --kernel-trace."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)
os.environ["M3S_ATTN_SPLITS"] = "1"
for (b, heads, sq, sk) in [(1, 16, 768, 64), (1, 16, 768, 256), (1, 16, 768, 768), (1, 16, 128, 768),
                           (1, 1, 768, 768), (1, 64, 768, 768), (4, 12, 768, 768)]:
    C = heads * 64
    q = torch.randn(b, sq, C, device=dev).bfloat16()
    kv = torch.randn(b, sk, 2 * C, device=dev).bfloat16()
    o = torch.empty(b, sq, C, device=dev, dtype=torch.bfloat16)
    for _ in range(20):
        ops.attn(q, C, sq * C, kv, kv[:, :, C:], 2 * C, sk * 2 * C, o, C, sq * C, b, heads, sq, sk)
    torch.cuda.synchronize()
    print("done", b, heads, sq, sk, flush=True)
