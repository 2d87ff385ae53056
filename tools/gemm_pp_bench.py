"""The product GEMM (libmonst3r_slam_amd m3s_vit_gemm) per tile configuration on the large
shapes: the table / heuristic choice, T256SQ (14), T256PP (15, the ping-pong kernel) and
hipBLASLt (torch.bmm, reference point only; on shapes it has run cleanly on this image),
interleaved rounds in one process.  Usage: python tools/gemm_pp_bench.py [MxNxKxB ...]"""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops

dev = torch.device("cuda:0")
ops = Ops(dev)
BLAS_OK = {(4096, 4096, 4096, 1), (8192, 8192, 8192, 1), (768, 6400, 7168, 2),
           (6144, 3072, 768, 4), (6144, 768, 3072, 4)}


def t_us(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


shapes = [(4096, 4096, 4096, 1), (8192, 8192, 8192, 1), (768, 6400, 7168, 2),
          (768, 7168, 1792, 2), (1536, 3072, 1024, 1), (1536, 4096, 1024, 1),
          (1536, 1024, 4096, 1), (6144, 3072, 768, 4), (6144, 768, 3072, 4),
          (6144, 3840, 768, 4), (6144, 768, 768, 4)]
if len(sys.argv) > 1:
    shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]
cfgs = [("table", None), ("T256SQ", "14"), ("T256PP", "15"), ("T192PP", "16")]
ORDERS = [o for o in os.environ.get("PP_ORDERS", "").split(",") if o]   # e.g. -4,-8,0
for o in ORDERS:
    cfgs.append((f"T256PP/o{o}", "15:" + o))
import ctypes
proto = None
pth = os.path.join(ROOT, "tools", "_build", "libgemm_pp_dev.so")
if os.path.exists(pth):   # the isolated main loop (tools/gemm_pp_dev.hip), same operands
    proto = ctypes.CDLL(pth)
    proto.pp_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 7 + \
        [ctypes.c_long] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
for (M, N, K, b) in shapes:
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(b, M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand(b, N, K, device=dev, generator=g) * 2 - 1).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    ref = torch.bmm(A.float(), B.float().transpose(1, 2))
    best, errs = {}, {}
    for rnd in range(3):
        for name, tile in cfgs:
            os.environ.pop("M3S_GEMM_ORDER", None)
            if tile is None:
                os.environ.pop("M3S_GEMM_TILE", None)
            else:
                os.environ["M3S_GEMM_TILE"] = tile.split(":")[0]
                if ":" in tile:
                    os.environ["M3S_GEMM_ORDER"] = tile.split(":")[1]
            fn = lambda: ops.gemm(A, B, C, M, N, K, b, sA=M * K, sB=N * K, sC=M * N)  # noqa
            best[name] = min(best.get(name, 1e30), t_us(fn))
            if rnd == 0:
                fn()
                torch.cuda.synchronize()
                errs[name] = float((C.float() - ref).abs().max() / ref.abs().max())
        if proto is not None:
            st = torch.cuda.current_stream().cuda_stream
            fn = lambda: proto.pp_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, b, K, K,  # noqa
                                       N, M * K, N * K, M * N, 4, 2, st)
            best["proto"] = min(best.get("proto", 1e30), t_us(fn))
            if rnd == 0:
                errs["proto"] = float((C.float() - ref).abs().max() / ref.abs().max())
    os.environ.pop("M3S_GEMM_TILE", None)
    os.environ.pop("M3S_GEMM_ORDER", None)
    tr = min(t_us(lambda: torch.bmm(A, B.transpose(1, 2))) for _ in range(3)) \
        if (M, N, K, b) in BLAS_OK else float("nan")
    fl = 2.0 * M * N * K * b
    line = " | ".join(f"{n} {t:7.1f} us {fl / t / 1e6:6.0f} TF/s (err {errs[n]:.1e})"
                      for n, t in best.items())
    print(f"{M}x{N}x{K}x{b}: {line} | hipBLASLt {tr:7.1f} us {fl / tr / 1e6:6.0f} TF/s",
          flush=True)
