"""Epilogue cost of the residual GEMMs (decoder / encoder fc2 and out-projections): the same
launch with the epilogue built up flag by flag — bf16 out, + bias + f32 out, + f32
residual, + LayerNorm-statistics producer (the 4137 set the model runs) — per tile
configuration.  Usage: python tools/gemm_epi_probe.py"""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops
from monst3r_slam_amd import _lib

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
        with torch.cuda.stream(s):
            e0.record(s); g.replay(); e1.record(s)
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


shapes = [("dec fc2 x4", 768, 768, 3072, 4), ("dec proj x4", 768, 768, 768, 4),
          ("enc fc2", 768, 1024, 4096, 1), ("enc proj", 768, 1024, 1024, 1)]
for name, M, N, K, b in shapes:
    A = (torch.rand(b, M, K, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(b, N, K, device=dev) * 0.1 - 0.05).bfloat16()
    bias = torch.rand(b, N, device=dev)
    C16 = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    C32 = torch.empty(b, M, N, device=dev)
    R = torch.rand(b, M, N, device=dev)
    xb = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    st = torch.empty(b, M, N // 128, 2, device=dev)
    fl = 2.0 * M * N * K * b
    common = dict(sA=M * K, sB=N * K, sC=M * N)
    variants = [
        ("bf16", lambda: ops.gemm(A, B, C16, M, N, K, b, **common)),
        ("+bias f32", lambda: ops.gemm(A, B, C32, M, N, K, b, bias=bias, sBias=N,
                                       flags=_lib.EPI_OUT_F32, **common)),
        ("+res", lambda: ops.gemm(A, B, C32, M, N, K, b, bias=bias, sBias=N, R=R, sR=M * N,
                                  flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, **common)),
        ("+stats", lambda: ops.gemm(A, B, C32, M, N, K, b, bias=bias, sBias=N, R=R, sR=M * N,
                                    flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32,
                                    ln_stats=(xb, st), **common)),
    ]
    for cfg in (0, 1, 2, 8, 12):
        if cfg:
            os.environ["M3S_GEMM_TILE"] = str(cfg)
            os.environ["M3S_GEMM_SPLITS"] = "1"
        else:
            os.environ.pop("M3S_GEMM_TILE", None)
            os.environ.pop("M3S_GEMM_SPLITS", None)
        row = [t_us(fn) for _, fn in variants]
        print(f"{name:12s} cfg {cfg:2d}: " + " | ".join(f"{v} {u:6.1f}" for (v, _), u in
                                                     zip(variants, row)) +
              f"  (full {fl / row[-1] / 1e6:5.0f} TF/s)", flush=True)
os.environ.pop("M3S_GEMM_TILE", None)
os.environ.pop("M3S_GEMM_SPLITS", None)
