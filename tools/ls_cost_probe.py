"""What the LN_STATS producer epilogue costs (round 6): the encoder fc2 shape
[1024, 1024, 4096] (and the decoder's [1024, 768, 3072] x 2) as a plain f32-residual GEMM,
+ LN_STATS with the bf16 copy, + LN_STATS with the shifted e4m3 copy — e4m3 and bf16
operands, graph-replayed, per-launch us."""
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
R32 = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32
for (M, N, K, b) in ((1024, 1024, 4096, 1), (1024, 768, 3072, 2), (1024, 1024, 1024, 1)):
    for f8 in (True, False):
        g = torch.Generator(device=dev).manual_seed(1)
        if f8:
            A = torch.randint(0, 100, (b, M, K), device=dev, dtype=torch.uint8, generator=g)
            B = torch.randint(0, 100, (b, N, K), device=dev, dtype=torch.uint8, generator=g)
            kw = dict(fp8=(torch.full((b, N), 1e-6, device=dev), N))
        else:
            A = (torch.randn(b, M, K, device=dev, generator=g) * 0.01).bfloat16()
            B = (torch.randn(b, N, K, device=dev, generator=g) * 0.01).bfloat16()
            kw = {}
        bias = torch.zeros(b, N, device=dev)
        x = torch.zeros(b, M, N, device=dev)
        st = torch.zeros(b, M, N // 128, 2, device=dev)
        xb = torch.zeros(b, M, N, device=dev, dtype=torch.bfloat16)
        xq = torch.zeros(b, M, N, device=dev, dtype=torch.uint8)
        sh = torch.zeros(b, N, device=dev)
        qs = torch.ones(b, device=dev)
        res = {}
        for tag, ls in (("plain", None), ("ls-bf16", (xb, st)), ("ls-e4m3", (xq, st, sh, qs))):
            def run():
                for _ in range(20):
                    ops.gemm(A, B, x, M, N, K, b, sA=M * K, sB=N * K, sC=M * N, sBias=N,
                             bias=bias, R=x, sR=M * N, flags=R32, ln_stats=ls, **kw)
            run()
            torch.cuda.synchronize()
            gph = bench.capture(run, dev)
            res[tag] = bench.time_replays(gph, dev, 10) / 20 * 1e3
        print(f"[{M},{N},{K},{b}] {'e4m3' if f8 else 'bf16'} operands: " +
              "  ".join(f"{k} {v:.2f} us" for k, v in res.items()), flush=True)
