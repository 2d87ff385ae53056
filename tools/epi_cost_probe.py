"""What the fused epilogues cost on the C4 chunk's decoder shapes (round 6): the same
[768, N, K] x 56 GEMM on the 256² ping-pong tile with bias only, + GELU, + the LayerNorm
fold, and the residual forms (f32 residual, + LN_STATS), graph-replayed, us per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)
Z, M = 56, 768
os.environ["M3S_GEMM_TILE"] = sys.argv[1] if len(sys.argv) > 1 else "15"
for N, K in ((3072, 768), (768, 768), (768, 3072)):
    g = torch.Generator(device=dev).manual_seed(1)
    A = (torch.randn(Z, M, K, device=dev, generator=g) * 0.5).bfloat16()
    B = (torch.randn(4, N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(4, N, device=dev, generator=g) * 0.1
    c1 = torch.randn(4, N, device=dev, generator=g)
    st = torch.rand(Z, M, K // 128, 2, device=dev, generator=g) + 0.5
    C = torch.empty(Z, M, N, device=dev, dtype=torch.bfloat16)
    x = torch.zeros(Z, M, N, device=dev)
    xb = torch.empty(Z, M, N, device=dev, dtype=torch.bfloat16)
    so = torch.empty(Z, M, N // 128, 2, device=dev)
    kw = dict(sA=M * K, sB=N * K, sC=M * N, sBias=N, wmod=4, bias=bias)
    cases = {"bias": dict(out=C), "gelu": dict(out=C, flags=_lib.EPI_GELU),
             "fold": dict(out=C, ln_fold=(st, c1, 0)),
             "fold+gelu": dict(out=C, flags=_lib.EPI_GELU, ln_fold=(st, c1, 0)),
             "f32": dict(out=x, flags=_lib.EPI_OUT_F32),
             "res": dict(out=x, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, R=x, sR=M * N),
             "res+stats": dict(out=x, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, R=x, sR=M * N,
                               ln_stats=(xb, so))}
    if K > 1024:   # the fold reads at most 8 groups of 128 (LayerNorm dim <= 1024)
        cases = {k: v for k, v in cases.items() if "fold" not in k}
    res = {}
    for tag, c in cases.items():
        c = dict(c)
        out = c.pop("out")

        def run():
            for _ in range(10):
                ops.gemm(A, B, out, M, N, K, Z, **kw, **c)
        run()
        torch.cuda.synchronize()
        gph = bench.capture(run, dev)
        res[tag] = bench.time_replays(gph, dev, 5) / 10 * 1e3
    fl = 2.0 * M * N * K * Z
    print(f"[{M},{N},{K}]x{Z} tile {os.environ['M3S_GEMM_TILE']}: " +
          "  ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f})" for k, v in res.items()), flush=True)
