"""Graph-timed refine_matches at 384x512 on a synthetic pair (tools only); M3S_LIB_PATH
selects an A/B build of the library.
Usage: [COHERENT=1] python tools/match_bench.py [batch] [jitter_px] [dilation_max]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
h, w, F = 384, 512, 24
n = h * w
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
J = int(sys.argv[2]) if len(sys.argv) > 2 else 4   # match jitter amplitude (px); 0 = smooth
DMAX = int(sys.argv[3]) if len(sys.argv) > 3 else 5  # dilation levels
g = torch.Generator(device=dev).manual_seed(0)
D11 = torch.nn.functional.normalize(torch.randn(B, h, w, F, device=dev, generator=g), dim=-1).half()
D21 = torch.nn.functional.normalize(torch.randn(B, n, F, device=dev, generator=g), dim=-1).half()
if os.environ.get("COHERENT"):
    # trained-network-like descriptors: a spatially smooth field (9 x 9 box filter of noise),
    # each query's descriptor its true match's plus noise — the coarse-to-fine search then
    # moves a tile's matches coherently toward the identity instead of scattering them
    f = torch.randn(B, F, h, w, device=dev, generator=g)
    f = torch.nn.functional.avg_pool2d(f, 9, stride=1, padding=4, count_include_pad=False)
    D11 = torch.nn.functional.normalize(f.permute(0, 2, 3, 1), dim=-1).half().contiguous()
    D21 = torch.nn.functional.normalize(D11.reshape(B, n, F).float() + 0.05 * torch.randn(
        B, n, F, device=dev, generator=g), dim=-1).half().contiguous()
# matches near the identity (as after iter_proj on consecutive frames): local windows overlap
yy, xx = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
jit = torch.randint(-J, J + 1, (B, 2, h, w), device=dev, generator=g) + (3 if J == 0 else 0)
p1 = torch.stack([(xx + jit[:, 0]).clamp(0, w - 1), (yy + jit[:, 1]).clamp(0, h - 1)], -1)
p1 = p1.reshape(B, n, 2).contiguous()
out = torch.empty_like(p1)


def refine():
    _lib.check(lib.m3s_refine_matches(_lib.ptr(D11), _lib.ptr(D21), _lib.ptr(p1), _lib.ptr(out), B,
                                      h, w, n, F, 3, DMAX, _lib.stream(dev)), "refine")


def graph_us(fn, rep=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(rep):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / rep


lib_tag = os.path.basename(os.environ.get("M3S_LIB_PATH", "") or "product") + (
    " coherent" if os.environ.get("COHERENT") else " random")
us = graph_us(refine)
print(f"refine_matches 384x512 r3 d{DMAX} b={B} jitter={J} [{lib_tag}]: {us:.1f} us "
      f"({us / B:.1f} us per pair)", flush=True)
