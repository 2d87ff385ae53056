"""Per-phase timeline of the GEMM kernel (s_memtime stamps, wave 0 of every workgroup):
prologue / vmcnt wait / barrier / MFMA phase per K-tile / epilogue in shader cycles, plus
s_memrealtime (100 MHz, chip-wide) at block start / end: the in-kernel clock (Δmemtime /
Δrealtime), each block's lifetime in µs, and the launch's block-start spread and span
against the HIP-event time.  Split-K blocks that exit after publishing their partial are
stamped too (column 'early').  Needs `make -C monst3r-slam_amd/csrc stamps`.
  python tools/gemm_stamps.py ["name,M,N,K,batch,tile,split,fused" ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402

lib = ctypes.CDLL(os.environ.get("M3S_STAMPS_LIB") or
                  os.path.join(ROOT, "monst3r-slam_amd/csrc/build/libm3s_gemm_stamps.so"))
lib.m3s_vit_gemm.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
lib.m3s_debug_set_stamps.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
W = 20
stamps = torch.zeros(W << 16, dtype=torch.int64, device=dev)
assert lib.m3s_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)


def gemm(A, B, C, M, N, K, b, tile, split, fused, bias):
    d = _lib.GemmDesc()
    d.A, d.lda, d.strideA = ctypes.c_void_p(A.data_ptr()), K, M * K
    d.B, d.ldb, d.strideB = ctypes.c_void_p(B.data_ptr()), K, N * K
    d.C, d.ldc, d.strideC = ctypes.c_void_p(C.data_ptr()), N, M * N
    d.bias, d.strideBias = ctypes.c_void_p(bias.data_ptr()), N
    d.M, d.N, d.K, d.batch, d.flags = M, N, K, b, _lib.EPI_BIAS
    d.workspace, d.workspace_bytes, d.split_k = ctypes.c_void_p(ws.data_ptr()), ws.numel(), split
    d.tile_counters, d.tile_counters_len = ctypes.c_void_p(cnt.data_ptr()), cnt.numel()
    os.environ["M3S_GEMM_TILE"] = str(tile)
    os.environ["M3S_GEMM_FUSED"] = str(fused)
    st = lib.m3s_vit_gemm(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == 0, st


shapes = [("enc fc2", 768, 1024, 4096, 1, 2, 1, 0), ("enc fc2", 768, 1024, 4096, 1, 10, 1, 0),
          ("enc fc2", 768, 1024, 4096, 1, 1, 1, 0), ("enc fc2", 768, 1024, 4096, 1, 1, 4, 0),
          ("enc fc2", 768, 1024, 4096, 1, 1, 4, 1), ("enc fc2", 768, 1024, 4096, 1, 2, 2, 0),
          ("enc proj", 768, 1024, 1024, 1, 2, 1, 0), ("enc proj", 768, 1024, 1024, 1, 1, 2, 0),
          ("enc fc1", 768, 4096, 1024, 1, 1, 1, 0), ("dec fc2", 768, 768, 3072, 4, 1, 1, 0),
          ("big", 4096, 4096, 4096, 1, 1, 1, 0), ("big", 4096, 4096, 4096, 1, 7, 1, 0)]
if len(sys.argv) > 1:   # "name,M,N,K,b,tile,split,fused" per argument
    shapes = [(a.split(",")[0], *[int(x) for x in a.split(",")[1:]]) for a in sys.argv[1:]]
for name, M, N, K, b, tile, split, fused in shapes:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = (torch.randn(b, N, K, device=dev) / K ** 0.5).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    bias = torch.randn(b, N, device=dev)
    for _ in range(200):                 # warm clocks and caches, back to back
        gemm(A, B, C, M, N, K, b, tile, split, fused, bias)
    stamps.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gemm(A, B, C, M, N, K, b, tile, split, fused, bias)
    e1.record()
    e1.synchronize()
    ev = e0.elapsed_time(e1) * 1e3
    s = stamps.view(-1, W).cpu()
    s = s[s[:, 6] > 0].double()
    nk = s[:, 5].clamp_min(1)
    rt = (s[:, 13] - s[:, 12]) / 100.0                     # µs per block (100 MHz)
    clk = s[:, 6] / rt / 1e3                               # GHz
    start = (s[:, 12] - s[:, 12].min()) / 100.0
    span = (s[:, 13].max() - s[:, 12].min()) / 100.0
    early = s[:, 14] > 0
    print(f"{name:8s} {M}x{N}x{K}x{b} tile {tile:2d} split {split} fused {fused}: event {ev:6.1f} us,"
          f" {len(s)} blocks ({int(early.sum())} early) | span {span:6.1f} us, start p50/p90/max "
          f"{start.quantile(0.5):5.1f}/{start.quantile(0.9):5.1f}/{start.max():5.1f} us | block "
          f"{rt.median():5.1f} us (p90 {rt.quantile(0.9):5.1f}) clk {clk.median():4.2f} GHz | cyc: "
          f"pro {s[:, 0].median():5.0f} wait/k {(s[:, 1] / nk).median():4.0f} bar/k "
          f"{(s[:, 2] / nk).median():4.0f} comp/k {(s[:, 3] / nk).median():5.0f} epi "
          f"{s[:, 4].median():5.0f} (out {s[:, 11].median():5.0f}) first-tile {s[:, 15].median():5.0f}"
          f" tail {s[:, 16].median():5.0f}", flush=True)
