"""Tile / split-K sweep of the fp8 (e4m3) GEMM path on the encoder/decoder shapes at
384x512 (S=768) and 512x512 (S=1024), against the bf16 kernel on the same shape.
Usage: python tools/fp8_tune.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd"), os.path.join(ROOT, "tools")]
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops, quant_e4m3  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)
REP = 20


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(REP):
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
        best = min(best, e0.elapsed_time(e1) * 1e3 / REP)
    return best


def main():
    shapes = []
    for S in (768, 1024):
        shapes += [(f"enc qkv S{S}", S, 3072, 1024, 1, 0), (f"enc proj S{S}", S, 1024, 1024, 1, 1),
                   (f"enc fc1 S{S}", S, 4096, 1024, 1, 2), (f"enc fc2 S{S}", S, 1024, 4096, 1, 1),
                   (f"dec qkv x4 S{S}", S, 2304, 768, 4, 0), (f"dec proj x4 S{S}", S, 768, 768, 4, 1),
                   (f"dec fc1 x4 S{S}", S, 3072, 768, 4, 2), (f"dec fc2 x4 S{S}", S, 768, 3072, 4, 1)]
    shapes += [("dec proj x2 S1024", 1024, 768, 768, 2, 1), ("dec fc2 x2 S1024", 1024, 768, 3072, 2, 1),
               ("big 4096^3", 4096, 4096, 4096, 1, 0)]
    cfgs = [(2, 1), (2, 2), (1, 1), (1, 2), (1, 4), (7, 1), (7, 2)]
    for name, M, N, K, b, kind in shapes:
        A = torch.randn(b, M, K, device=dev).clamp(-8, 8).to(torch.float8_e4m3fn).view(torch.uint8)
        Bq, sc = quant_e4m3(torch.randn(b, N, K, device=dev) / K ** 0.5)
        Ab = torch.randn(b, M, K, device=dev).bfloat16()
        Bb = (torch.randn(b, N, K, device=dev) / K ** 0.5).bfloat16()
        bias = torch.randn(b, N, device=dev)
        if kind == 1:
            C = torch.zeros(b, M, N, device=dev)
            flags, R, o8 = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32, C, False
        elif kind == 2:
            C = torch.empty(b, M, N, device=dev, dtype=torch.uint8)
            flags, R, o8 = _lib.EPI_GELU, None, True
        else:
            C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
            flags, R, o8 = 0, None, False
        Cb = torch.empty(b, M, N, device=dev, dtype=torch.float32 if kind == 1 else torch.bfloat16)
        fl = 2.0 * M * N * K * b

        def f8(split):
            return lambda: ops.gemm(A, Bq, C, M, N, K, b, sA=M * K, sB=N * K, sC=M * N, bias=bias,
                                    sBias=N, R=R, sR=M * N, flags=flags, split_k=split,
                                    fp8=(sc, N), out_fp8=o8)
        os.environ["M3S_GEMM_TILE"] = "0"
        auto = graph_us(f8(0))
        bfl = graph_us(lambda: ops.gemm(Ab, Bb, Cb, M, N, K, b, sA=M * K, sB=N * K, sC=M * N,
                                        bias=bias, sBias=N, R=Cb if kind == 1 else None, sR=M * N,
                                        flags=flags if kind != 2 else _lib.EPI_GELU))
        line = f"{name:22s} {M}x{N}x{K}x{b} auto {auto:6.1f}us {fl / auto / 1e6:5.0f}TF bf16 {bfl:6.1f}us |"
        for tile, split in cfgs:
            os.environ["M3S_GEMM_TILE"] = str(tile)
            try:
                us = graph_us(f8(split))
                line += f" t{tile}s{split} {us:6.1f}"
            except RuntimeError:
                line += f" t{tile}s{split}  n/a "
        os.environ["M3S_GEMM_TILE"] = "0"
        print(line, flush=True)


if __name__ == "__main__":
    main()
