"""DMA-ring depth sweep: the pair's M = 768 GEMM shapes under each tile config
(M3S_GEMM_TILE), back-to-back launches timed with HIP events (no split-K unless the
default heuristic picks it: tile 0)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops  # noqa: E402
from monst3r_slam_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)


def t_us(fn, n=30):
    """n launches captured back-to-back in a HIP graph (eager launches are host-bound)."""
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / (3 * n) * 1e3


shapes = [("enc qkv", 768, 3072, 1024, 1, 0), ("enc proj", 768, 1024, 1024, 1, 1),
          ("enc fc1", 768, 4096, 1024, 1, 0), ("enc fc2", 768, 1024, 4096, 1, 1),
          ("dec qkv", 768, 2304, 768, 4, 0), ("dec proj", 768, 768, 768, 4, 1),
          ("dec fc1", 768, 3072, 768, 4, 0), ("dec fc2", 768, 768, 3072, 4, 1),
          ("dec kv", 768, 1536, 768, 4, 0), ("big", 4096, 4096, 4096, 1, 0)]
tiles = [int(t) for t in os.environ.get("TILES", "0,1,10,11,2,12,7").split(",")]
for name, M, N, K, b, res in shapes:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = torch.randn(b, N, K, device=dev).bfloat16()
    bias = torch.randn(b * N, device=dev)
    ref = torch.bmm(A.float(), B.float().transpose(1, 2)) + bias.view(b, 1, N)
    if res:
        R = torch.randn(b, M, N, device=dev)
        C = torch.empty(b, M, N, device=dev)
        kw = dict(R=R, sR=M * N, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32)
        ref = ref + R
    else:
        C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
        kw = dict(flags=_lib.EPI_GELU)
        ref = torch.nn.functional.gelu(ref)
    fl = 2.0 * M * N * K * b
    out = []
    for t in tiles:
        os.environ["M3S_GEMM_TILE"] = str(t)
        sk = 0 if t == 0 else 1
        C.zero_()
        us = t_us(lambda: ops.gemm(A, B, C, M, N, K, b, sA=M * K, sB=N * K, sC=M * N, bias=bias,
                                   sBias=N, split_k=sk, **kw))
        err = float((C.float() - ref).abs().max() / ref.abs().max())
        out.append(f"t{t}:{us:6.1f}us/{fl / us / 1e6:5.0f}TF" + ("" if err < 1e-2 else f" BAD{err:.1e}"))
    os.environ.pop("M3S_GEMM_TILE", None)
    print(f"{name:9s} {M}x{N}x{K}x{b}: " + "  ".join(out), flush=True)
