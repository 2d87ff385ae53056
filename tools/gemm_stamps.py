"""Per-phase timeline of the GEMM kernel (s_memtime stamps, wave 0 of every workgroup):
prologue / vmcnt wait / barrier / MFMA phase per K-tile / epilogue, in shader cycles.
Needs `make -C monst3r-slam_amd/csrc stamps`."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "monst3r-slam_amd/csrc/build/libm3s_gemm_stamps.so"))
lib.m3s_vit_gemm.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
lib.m3s_debug_set_stamps.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
stamps = torch.zeros(12 << 16, dtype=torch.int64, device=dev)
assert lib.m3s_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)


def gemm(A, B, C, M, N, K, b, tile, split, flags=0, R=None):
    d = _lib.GemmDesc()
    d.A, d.lda, d.strideA = ctypes.c_void_p(A.data_ptr()), K, M * K
    d.B, d.ldb, d.strideB = ctypes.c_void_p(B.data_ptr()), K, N * K
    d.C, d.ldc, d.strideC = ctypes.c_void_p(C.data_ptr()), N, M * N
    d.R, d.ldr, d.strideR = (ctypes.c_void_p(R.data_ptr()) if R is not None else None), N, M * N
    d.M, d.N, d.K, d.batch, d.flags = M, N, K, b, flags
    d.workspace, d.workspace_bytes, d.split_k = ctypes.c_void_p(ws.data_ptr()), ws.numel(), split
    os.environ["M3S_GEMM_TILE"] = str(tile)
    st = lib.m3s_vit_gemm(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == 0, st


shapes = [("enc fc1", 768, 4096, 1024, 1, 1, 1), ("enc fc1 S4", 768, 4096, 1024, 1, 10, 1),
          ("enc fc1 S5", 768, 4096, 1024, 1, 11, 1),
          ("dec fc2", 768, 768, 3072, 4, 1, 1), ("dec fc2 S5", 768, 768, 3072, 4, 11, 1),
          ("dec fc1", 768, 3072, 768, 4, 1, 1), ("dec fc1 S5", 768, 3072, 768, 4, 11, 1),
          ("big", 4096, 4096, 4096, 1, 1, 1), ("big S5", 4096, 4096, 4096, 1, 11, 1)]
for name, M, N, K, b, tile, split in shapes:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = torch.randn(b, N, K, device=dev).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        stamps.zero_()
        gemm(A, B, C, M, N, K, b, tile, split)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gemm(A, B, C, M, N, K, b, tile, split)
    e1.record()
    e1.synchronize()
    s = stamps.view(-1, 12).cpu()
    s = s[s[:, 6] > 0].double()
    nk = s[:, 5]
    t0 = s[:, 7]
    span = (s[:, 7] + s[:, 6]).max() - t0.min()
    print(f"{name:9s} {M}x{N}x{K}x{b} tile {tile}: {e0.elapsed_time(e1) * 1e3:7.1f} us, "
          f"{len(s)} blocks | per block: prologue {s[:, 0].mean():6.0f} "
          f"wait/step {(s[:, 1] / nk).mean():6.0f} bar/step {(s[:, 2] / nk).mean():6.0f} "
          f"comp/step {(s[:, 3] / nk).mean():6.0f} epi {s[:, 4].mean():6.0f} total "
          f"{s[:, 6].mean():7.0f} | epi: prefetch {s[:, 8].mean():5.0f} sync1 {s[:, 9].mean():5.0f} "
          f"lds+sync2 {s[:, 10].mean():5.0f} out {s[:, 11].mean():5.0f}", flush=True)
    # s_memtime is per XCD: spans only within one XCD's blocks (block b → XCD b % 8)
    bid = torch.arange(stamps.view(-1, 12).shape[0])[stamps.view(-1, 12)[:, 6].cpu() > 0]
    sp, sps = [], []
    for x in range(8):
        m = (bid % 8) == x
        if m.any():
            sx, ex = t0[m], t0[m] + s[m, 6]
            sp.append(float(ex.max() - sx.min()))
            sps.append(float((sx - sx.min()).quantile(0.9)))
    ev = e0.elapsed_time(e1) * 1e3
    print(f"          per-XCD span {sum(sp) / len(sp):8.0f} cyc (max {max(sp):8.0f}) → "
          f"{max(sp) / ev:5.0f} cyc/us vs event {ev:6.1f} us | start p90 {sum(sps) / len(sps):6.0f}"
          f" | block total p10 {s[:, 6].quantile(0.1):6.0f} p90 {s[:, 6].quantile(0.9):6.0f}",
          flush=True)
