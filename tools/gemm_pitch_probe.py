"""Row-pitch probe: the skinny M = 768 GEMMs with operand rows padded past a power-of-two
byte stride (A / B row pitch K + pad elements), to test L2 channel camping of the LDS-DMA
K-slices (all rows of a tile's K-slice at one 2^n stride).
  python tools/gemm_pitch_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd"), os.path.join(ROOT, "tools")]
from gemm_split_probe import timed, ops, dev  # noqa: E402
from monst3r_slam_amd import _lib  # noqa: E402


def main():
    for (M, N, K, b) in ((768, 1024, 4096, 1), (768, 1024, 1024, 1), (768, 4096, 1024, 1),
                         (768, 768, 3072, 4), (768, 3072, 768, 4), (4096, 4096, 4096, 1)):
        for tile in ("0", "2", "10", "1", "11"):
            res = []
            for pad in (0, 64, 128, 256):
                A = torch.randn(b, M, K + pad, device=dev).bfloat16()
                B = (torch.randn(b, N, K + pad, device=dev) / K ** 0.5).bfloat16()
                C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
                bias = torch.randn(b, N, device=dev)
                os.environ["M3S_GEMM_TILE"] = tile
                os.environ["M3S_GEMM_SPLITS"] = "1"
                if tile == "0":
                    os.environ.pop("M3S_GEMM_TILE")
                    os.environ.pop("M3S_GEMM_SPLITS")
                us = timed(lambda: ops.gemm(A, B, C, M, N, K, b, lda=K + pad, ldb=K + pad,
                                            sA=M * (K + pad), sB=N * (K + pad), sC=M * N,
                                            bias=bias, sBias=N, flags=_lib.EPI_BIAS))
                res.append(f"pad {pad:3d}: {us:7.2f} us {2.0 * M * N * K * b / us / 1e6:6.1f} TF/s")
            print(f"{M}x{N}x{K}x{b} tile {tile:>2s} | " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
