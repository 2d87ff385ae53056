"""LN_STATS shifted e4m3 copy probe (round 6 debugging): per tile configuration and
problem, the ratio of the kernel's copy to (x − shift)·qscale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)
for M, N, K, batch in ((768, 768, 1024, 4), (768, 768, 1024, 2), (256, 256, 256, 1)):
    for tile in ("0", "2", "7", "12"):
        if tile == "0":
            os.environ.pop("M3S_GEMM_TILE", None)
        else:
            os.environ["M3S_GEMM_TILE"] = tile
        g = torch.Generator(device=dev).manual_seed(31)
        A = torch.randn(batch, M, K, device=dev, generator=g).bfloat16()
        B = (torch.randn(2, N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
        bias = torch.randn(2, N, device=dev, generator=g)
        x = torch.randn(batch, M, N, device=dev, generator=g)
        shift = torch.zeros(2, N, device=dev)
        qs = torch.tensor([1.0, 1.0], device=dev)
        xq = torch.zeros(batch, M, N, device=dev, dtype=torch.uint8)
        st = torch.zeros((batch, M, N // 128, 2), device=dev)
        ops.gemm(A, B, x, M, N, K, batch, sA=M * K, sB=N * K, sC=M * N, sBias=N, wmod=2,
                 bias=bias, R=x, sR=M * N, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32,
                 ln_stats=(xq, st, shift, qs))
        torch.cuda.synchronize()
        q = xq.view(torch.float8_e4m3fn).float()
        r = x.clamp(-448, 448).to(torch.float8_e4m3fn).float()
        bad = (q != r)
        print(M, N, K, batch, "tile", tile, "mismatch frac per problem",
              [round(float(bad[z].float().mean()), 4) for z in range(batch)],
              "ratio med", [round(float((q[z] / r[z]).nanmedian()), 3) for z in range(batch)])
        if bad.any():
            idx = bad.nonzero()[:4].tolist()
            print("   first bad", idx, [(float(q[tuple(i)]), float(r[tuple(i)])) for i in idx])
