"""Graph-timed refine_matches / iter_proj at 384x512 on a synthetic pair (tools only)."""
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
g = torch.Generator(device=dev).manual_seed(0)
D11 = torch.nn.functional.normalize(torch.randn(B, h, w, F, device=dev, generator=g), dim=-1).half()
D21 = torch.nn.functional.normalize(torch.randn(B, n, F, device=dev, generator=g), dim=-1).half()
# matches near the identity (as after iter_proj on consecutive frames): local windows overlap
yy, xx = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
jit = torch.randint(-J, J + 1, (B, 2, h, w), device=dev, generator=g) + (3 if J == 0 else 0)
p1 = torch.stack([(xx + jit[:, 0]).clamp(0, w - 1), (yy + jit[:, 1]).clamp(0, h - 1)], -1)
p1 = p1.reshape(B, n, 2).contiguous()
out = torch.empty_like(p1)


def refine():
    _lib.check(lib.m3s_refine_matches(_lib.ptr(D11), _lib.ptr(D21), _lib.ptr(p1), _lib.ptr(out), B,
                                      h, w, n, F, 3, 5, _lib.stream(dev)), "refine")


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


D11p = torch.empty((B, 3, n, 8), dtype=torch.float16, device=dev)
out2 = torch.empty_like(p1)


def planar():
    _lib.check(lib.m3s_desc_planar(_lib.ptr(D11), _lib.ptr(D11p), B, n, _lib.stream(dev)), "pl")


def refine_planar():
    _lib.check(lib.m3s_refine_matches_planar(_lib.ptr(D11p), _lib.ptr(D21), _lib.ptr(p1),
                                             _lib.ptr(out2), B, h, w, 3, 5, _lib.stream(dev)),
               "refine_planar")


tag = os.environ.get("M3S_REFINE_KERNEL", "r3")
us = graph_us(refine)
print(f"refine_matches 384x512 r3 d5 b={B} jitter={J} {tag}: {us:.1f} us ({us / B:.1f} us per pair)", flush=True)
us = graph_us(planar)
print(f"desc_planar 384x512 b={B}: {us:.1f} us", flush=True)
us = graph_us(refine_planar)
print(f"refine_matches_planar 384x512 r3 d5 b={B} jitter={J}: {us:.1f} us ({us / B:.1f} us per pair)",
      flush=True)
torch.cuda.synchronize()
print("planar == rows:", bool(torch.equal(out, out2)), flush=True)
