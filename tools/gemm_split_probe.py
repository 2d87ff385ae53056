"""Split-K probe for the skinny M = 768 GEMMs (encoder fc2 / out-proj): per (tile config,
splits, fused) the graph-replayed time of 20 back-to-back launches, plain bias epilogue and
the LN_STATS residual producer.  Run under rocprofv3 --kernel-trace --stats to separate the
main kernel from splitk_reduce_kernel.
  python tools/gemm_split_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)


def timed(fn, reps=20):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            g.replay()
        e1.record(s)
        e1.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    only = None
    if len(sys.argv) > 1:   # e.g. "1:1:0,1:4:0" = (tile, splits, fused) list, fc2 shape, bias
        only = [tuple(int(v) for v in c.split(":")) for c in sys.argv[1].split(",")]
    for (M, N, K) in ((768, 1024, 4096), (768, 1024, 1024)):
        if only and K != 4096:
            continue
        A = torch.randn(M, K, device=dev).bfloat16()
        B = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        bias = torch.randn(N, device=dev)
        x = torch.randn(M, N, device=dev)
        C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(M, N // 128, 2, device=dev)
        for epi in (("bias",) if only else ("bias", "ln_stats")):
            def run():
                if epi == "bias":
                    ops.gemm(A, B, C2, M, N, K, bias=bias, flags=_lib.EPI_BIAS)
                else:
                    ops.gemm(A, B, x, M, N, K, bias=bias, R=x, ln_stats=(C2, stats),
                             flags=_lib.EPI_BIAS | _lib.EPI_RES_F32 | _lib.EPI_OUT_F32)
            for tile in (2, 10, 1, 11, 7):
                for sp in (1, 2, 3, 4, 6, 8):
                    for fu in ((0, 1) if sp > 1 else (0,)):
                        if only and (tile, sp, fu) not in only:
                            continue
                        os.environ.update(M3S_GEMM_TILE=str(tile), M3S_GEMM_SPLITS=str(sp),
                                          M3S_GEMM_FUSED=str(fu))
                        try:
                            us = timed(run)
                        except Exception as e:  # noqa: BLE001
                            print(f"{M}x{N}x{K} {epi} tile {tile} split {sp} fused {fu}: {e}")
                            continue
                        fl = 2.0 * M * N * K
                        print(f"{M}x{N}x{K} {epi:8s} tile {tile:2d} split {sp} fused {fu}: "
                              f"{us:7.2f} us {fl / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
