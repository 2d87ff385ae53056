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
          ("dec kv", 768, 1536, 768, 4, 0), ("dec qkvkv", 768, 3840, 768, 4, 0),
          ("big", 4096, 4096, 4096, 1, 0)]
tiles = [int(t) for t in os.environ.get("TILES", "0,1,2,7,8").split(",")]
# DPT implicit 3x3 convs (NHWC bf16, Z = 4): (name, H, W, cin, cout, epilogue)
convs = [("head.2+dpt", 384, 512, 128, 128, "dpt"), ("head.0", 192, 256, 256, 128, "bias"),
         ("rcu 96x128", 96, 128, 256, 256, "relu_res"), ("rn0 96x128", 96, 128, 96, 256, "none"),
         ("rcu 48x64", 48, 64, 256, 256, "relu_res")]
for name, H, W, cin, cout, epi in convs if os.environ.get("CONVS", "1") != "0" else []:
    b = 4
    x = torch.randn(b, H, W, cin, device=dev).bfloat16()
    w = (torch.randn(cout, 9 * cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
    bias = torch.randn(cout, device=dev)
    out = torch.empty(b, H, W, cout, device=dev, dtype=torch.bfloat16)
    kw = dict(sA=H * W * cin, sB=0, sC=H * W * cout, conv=(H, W, cin, H, W, 1))
    if epi == "dpt":
        w4, b4 = torch.randn(1, 4, 128, device=dev) * 0.05, torch.zeros(1, 4, device=dev)
        pts = torch.empty(b, H * W, 3, device=dev)
        conf = torch.empty(b, H * W, device=dev)
        kw.update(bias=bias, flags=_lib.EPI_RELU, dpt=(w4, b4, pts, conf, 1.0), wmod=1)
    elif epi == "bias":
        kw.update(bias=bias)
    elif epi == "relu_res":
        R = torch.randn(b, H, W, cout, device=dev).bfloat16()
        kw.update(bias=bias, R=R, sR=H * W * cout, flags=_lib.PRO_RELU | _lib.EPI_RES_BF16)
    fl = 2.0 * H * W * cout * 9 * cin * b
    res_s = []
    for t in tiles:
        os.environ["M3S_GEMM_TILE"] = str(t)
        us = t_us(lambda: ops.gemm(x, w, out, H * W, cout, 9 * cin, b, **kw), n=10)
        res_s.append(f"t{t}:{us:7.1f}us/{fl / us / 1e6:5.0f}TF")
    os.environ.pop("M3S_GEMM_TILE", None)
    print(f"conv {name:11s} {H}x{W} {cin}->{cout} x{b}: " + "  ".join(res_s), flush=True)
for name, M, N, K, b, res in shapes if os.environ.get("GEMMS", "1") != "0" else []:
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
