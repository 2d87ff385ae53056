"""What bounds the M = 768 GEMMs: the same launches with one or both operands made
cache-hot (lda = 0 / ldb = 0: every row of the operand is the same 128-B-per-K-step row,
so its DMA always hits L1/L2) against the real operands.  If 'both hot' runs near the
MFMA time, the normal launch is bound by where its bytes come from (L2 misses / fabric);
if not, by the block's own issue structure.  Usage: python tools/gemm_locality_probe.py"""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops

dev = torch.device("cuda:0")
ops = Ops(dev)


def t_us(fn, n=30, reps=3):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):  # replay() launches on the current stream
            e0.record(s); g.replay(); e1.record(s)
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


shapes = [("enc fc2", 768, 1024, 4096, 1), ("enc proj", 768, 1024, 1024, 1),
          ("enc qkv", 768, 3072, 1024, 1), ("dec fc2 x4", 768, 768, 3072, 4),
          ("dec fc1 x4", 768, 3072, 768, 4), ("big 4096^3", 4096, 4096, 4096, 1)]
cfgs = [(10, 1), (1, 1), (2, 1), (12, 1), (1, 4), (2, 4)]
for name, M, N, K, b in shapes:
    A = (torch.rand(b, M, K, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(b, N, K, device=dev) * 2 - 1).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K * b
    for cfg, sp in cfgs:
        if name.startswith("big") and sp > 1:
            continue
        os.environ["M3S_GEMM_TILE"] = str(cfg)
        os.environ["M3S_GEMM_SPLITS"] = str(sp)
        row = []
        for la, lb in ((K, K), (0, K), (K, 0), (0, 0)):
            us = t_us(lambda: ops.gemm(A, B, C, M, N, K, b, lda=la, ldb=lb, sA=M * K if la else 0,
                                       sB=N * K if lb else 0, sC=M * N))
            row.append(us)
        print(f"{name:11s} {M}x{N}x{K}x{b} cfg {cfg:2d} split {sp}: normal {row[0]:7.1f} us "
              f"({fl / row[0] / 1e6:6.1f} TF/s) | A hot {row[1]:7.1f} | B hot {row[2]:7.1f} | "
              f"both hot {row[3]:7.1f} ({fl / row[3] / 1e6:6.1f} TF/s)", flush=True)
os.environ.pop("M3S_GEMM_TILE", None)
os.environ.pop("M3S_GEMM_SPLITS", None)
