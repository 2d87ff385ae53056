"""Tile / split-K sweep of the HIP GEMM on the pair-inference shapes (graph-replayed so the
Python launch cost is not in the timing).  torch (hipBLASLt / MIOpen) as a reference point.
Usage: python tools/gemm_tune.py [--quick]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

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


def run(label, fl, fn_for, cfgs, ref=None):
    res = []
    for tile, split in cfgs:
        os.environ["M3S_GEMM_TILE"] = str(tile)
        try:
            us = graph_us(fn_for(split))
        except RuntimeError as ex:  # config not applicable
            res.append(((tile, split), None, str(ex)[:40]))
            continue
        res.append(((tile, split), us, ""))
    os.environ["M3S_GEMM_TILE"] = "0"
    us_auto = graph_us(fn_for(0))
    line = f"{label:34s} auto {us_auto:7.1f}us {fl / us_auto / 1e6:6.0f}TF |"
    for (tile, split), us, err in res:
        line += f" t{tile}s{split} " + (f"{us:6.1f}" if us else "  n/a ")
    if ref is not None:
        ur = graph_us(ref)
        line += f" | torch {ur:6.1f}us {fl / ur / 1e6:6.0f}TF"
    print(line, flush=True)


quick = "--quick" in sys.argv
gemms = [("enc qkv", 768, 3072, 1024, 1, 0), ("enc proj", 768, 1024, 1024, 1, 1),
         ("enc fc1", 768, 4096, 1024, 1, 2), ("enc fc2", 768, 1024, 4096, 1, 1),
         ("dec qkv x4", 768, 2304, 768, 4, 0), ("dec proj x4", 768, 768, 768, 4, 1),
         ("dec kv x4", 768, 1536, 768, 4, 0), ("dec fc1 x4", 768, 3072, 768, 4, 2),
         ("dec fc2 x4", 768, 768, 3072, 4, 1), ("dec embed x4", 768, 768, 1024, 4, 0),
         ("lf fc1 x2", 768, 7168, 1792, 2, 2), ("lf fc2 x2", 768, 6400, 7168, 2, 0),
         ("ap0 x4", 768, 96, 1024, 4, 0), ("ap0t x4", 768, 1536, 96, 4, 0),
         ("big 4096^3", 4096, 4096, 4096, 1, 0)]
for name, M, N, K, b, kind in gemms:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = (torch.randn(b, N, K, device=dev) / K ** 0.5).bfloat16()
    bias = torch.randn(b, N, device=dev)
    if kind == 1:  # f32 residual stream update
        C = torch.zeros(b, M, N, device=dev)
        flags = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32
        R = C
    else:
        C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
        flags = _lib.EPI_GELU if kind == 2 else 0
        R = None

    def fn_for(split, A=A, B=B, C=C, M=M, N=N, K=K, b=b, flags=flags, R=R, bias=bias):
        return lambda: ops.gemm(A, B, C, M, N, K, b, sA=M * K, sB=N * K, sC=M * N, bias=bias,
                                sBias=N, R=R, sR=M * N, flags=flags, split_k=split)
    cfgs = [(1, 1), (2, 1), (7, 1), (8, 1), (9, 1), (8, 2)] if quick else [(1, 1), (1, 2), (1, 4), (2, 1), (2, 2), (4, 1), (4, 2),
                                           (5, 1), (5, 2), (6, 1), (6, 2), (6, 4)]
    run(f"{name} {M}x{N}x{K}x{b}", 2.0 * M * N * K * b, fn_for, cfgs,
        ref=lambda A=A, B=B: torch.bmm(A, B.transpose(1, 2)))

convs = [("head.2", 384, 512, 128, 128, 4), ("head.0", 192, 256, 256, 128, 4),
         ("rcu r1", 192, 256, 256, 256, 4), ("rcu r2", 96, 128, 256, 256, 4),
         ("rcu r3", 48, 64, 256, 256, 4), ("rcu r4", 24, 32, 256, 256, 4),
         ("layer1_rn", 96, 128, 96, 256, 4), ("layer2_rn", 48, 64, 192, 256, 4),
         ("ap3 s2", 24, 32, 1024, 1024, 4)]
for name, H, W, cin, cout, b in convs:
    st = 2 if "s2" in name else 1
    Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
    x = torch.randn(b, H, W, cin, device=dev).bfloat16()
    w = (torch.randn(cout, 9 * cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
    out = torch.empty(b, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)

    def fn_for(split, x=x, w=w, out=out, H=H, W=W, cin=cin, cout=cout, b=b, st=st, Ho=Ho, Wo=Wo):
        return lambda: ops.gemm(x, w, out, Ho * Wo, cout, 9 * cin, b, sA=H * W * cin, sB=0,
                                sC=Ho * Wo * cout, conv=(H, W, cin, Ho, Wo, st), flags=_lib.PRO_RELU)
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wn = w.reshape(cout, 3, 3, cin).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    run(f"conv {name} {H}x{W} {cin}->{cout} x{b}", 2.0 * Ho * Wo * cout * 9 * cin * b, fn_for,
        [(1, 1), (2, 1), (6, 1), (7, 1)] if quick else [(1, 1), (2, 1), (3, 1), (6, 1), (7, 1)],
        ref=lambda xn=xn, wn=wn, st=st: torch.nn.functional.conv2d(xn, wn, padding=1, stride=st))

# attention (encoder: 1 x 16 heads, decoder: 4 x 12 heads; 768 tokens, head dim 64)
for name, b, heads in [("attn enc", 1, 16), ("attn dec x4", 4, 12)]:
    S, C = 768, heads * 64
    qkv = torch.randn(b, S, 3 * C, device=dev).bfloat16()
    o = torch.empty(b, S, C, device=dev, dtype=torch.bfloat16)
    us_aw = {}
    for aw in ("2", "4"):
        os.environ["M3S_ATTN_AW"] = aw
        us_aw[aw] = graph_us(lambda: ops.attn(qkv, 3 * C, S * 3 * C, qkv[:, :, C:], qkv[:, :, 2 * C:],
                                              3 * C, S * 3 * C, o, C, S * C, b, heads, S, S))
    del os.environ["M3S_ATTN_AW"]
    us = graph_us(lambda: ops.attn(qkv, 3 * C, S * 3 * C, qkv[:, :, C:], qkv[:, :, 2 * C:], 3 * C,
                                   S * 3 * C, o, C, S * C, b, heads, S, S))
    print(f"{name} AW=2 {us_aw['2']:.1f}us AW=4 {us_aw['4']:.1f}us")
    qh = qkv.reshape(b, S, 3, heads, 64).permute(2, 0, 3, 1, 4).contiguous()
    ur = graph_us(lambda: torch.nn.functional.scaled_dot_product_attention(qh[0], qh[1], qh[2]))
    fl = 4.0 * S * S * 64 * heads * b
    print(f"{name:34s} hip {us:7.1f}us {fl / us / 1e6:6.0f}TF | torch sdpa {ur:7.1f}us "
          f"{fl / ur / 1e6:6.0f}TF", flush=True)
