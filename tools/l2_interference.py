"""What slows a decoder-shaped GEMM inside the C3 step?  (tools only, round 5)

One GEMM shape launched REP times on stream s1, each launch's own span taken from the step
timeline's in-kernel stamps (m3s_timeline_set: first block start .. last wave end), under:
  alone   back to back (operands hot in L2 / MALL from the previous launch)
  cold    a 512 MB fill between launches on s1 (operands evicted from L2 and the 256 MB MALL,
          as in the step, where ~1.2 GB of weights stream per frame)
  tiny    beside a graph of tiny one-block kernels on s2 (nothing but launches: the
          dispatch acquire / release fences)
  spin    beside one single-thread spin kernel on s2 (a CU taken, no launches)
  heavy   beside a chain of 4096x4096x1024 GEMMs on s2 (the chip shared with MFMA work)
  heavy+cold
Usage: python tools/l2_interference.py [M N K batch]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
args = [int(a) for a in sys.argv[1:]]
M, N, K, B = args[:4] if len(args) >= 4 else (768, 768, 3072, 2)
REP = 24
ops = Ops(dev)
lib, P = _lib.load(), _lib.ptr
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(B, M, K, device=dev, generator=g).bfloat16()
W = torch.randn(B, N, K, device=dev, generator=g).bfloat16()
C = torch.empty(B, M, N, device=dev, dtype=torch.bfloat16)
tiny = torch.zeros(256, device=dev)
flush = torch.empty(128 << 20, device=dev)           # 512 MB
HA = torch.randn(4096, 1024, device=dev, generator=g).bfloat16()
HB = torch.randn(4096, 1024, device=dev, generator=g).bfloat16()
HC = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
cap_slots = 256
slot = torch.empty((cap_slots, 132), dtype=torch.int64, device=dev)
tl = slot[:, :128].view(cap_slots, 64, 2)
slot[:, 128:] = 0
nlog = 1 << 16
blog = torch.zeros((nlog, 8), dtype=torch.int64, device=dev)
bcnt = torch.zeros(2, dtype=torch.int32, device=dev)
slot[:, 128] = blog.data_ptr()
slot[:, 129] = bcnt.data_ptr()
slot[:, 130] = nlog


def capture(fn, st, timeline=False):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    if timeline:
        _lib.check(lib.m3s_timeline_set(P(slot), cap_slots), "timeline_set")
        slot[:, 128] = blog.data_ptr()      # the headers, zeroed by the set
        slot[:, 129] = bcnt.data_ptr()
        slot[:, 130] = nlog
    try:
        with torch.cuda.graph(gr, stream=st):
            fn()
    finally:
        if timeline:
            lib.m3s_timeline_set(None, 0)
    torch.cuda.synchronize()
    return gr


def chain(cold):
    def fn():
        for _ in range(REP):
            if cold:
                flush.fill_(1.0)
            ops.gemm(A, W, C, M, N, K, B, sA=M * K, sB=N * K, sC=M * N)
    return fn


def heavy():
    for _ in range(60):
        ops.gemm(HA, HB, HC, 4096, 4096, 1024, 1)


def tinies():
    for _ in range(3000):
        tiny.add_(1.0)


graphs = {"hot": capture(chain(False), s1, True), "cold": capture(chain(True), s1, True)}
g_heavy, g_tiny = capture(heavy, s2), capture(tinies, s2)


phases = {}


def run(which, other, name=None):
    tl[..., 0] = -1
    tl[..., 1] = 0
    bcnt.zero_()
    torch.cuda.synchronize()
    if other is not None:
        with torch.cuda.stream(s2):
            if other == "spin":
                torch.cuda._sleep(int(5e6))
            else:
                (g_heavy if other == "heavy" else g_tiny).replay()
    with torch.cuda.stream(s1):
        graphs[which].replay()
    torch.cuda.synchronize()
    lg = blog[:min(int(bcnt[0]), nlog)].cpu().numpy().astype(np.float64)
    ph = lg[:, 4:8]
    ok = (ph > 0).all(1)
    x, ph = lg[ok], ph[ok]
    if name is not None and len(x):
        phases[name] = ((x[:, 1] - x[:, 0]).mean() * 1e-2, (ph[:, 0] - x[:, 0]).mean() * 1e-2,
                        (ph[:, 1] - ph[:, 0]).mean() * 1e-2, (ph[:, 2] - ph[:, 1]).mean() * 1e-2,
                        (x[:, 1] - ph[:, 2]).mean() * 1e-2)
    t = tl[:REP].cpu().numpy()
    st = np.where(t[..., 0] > 0, t[..., 0], np.iinfo(np.int64).max).min(1)
    en = t[..., 1].max(1)
    return float(np.median((en - st)[2:]) * 1e-2)    # us; first launches dropped


cases = [("alone", "hot", None), ("cold", "cold", None), ("tiny", "hot", "tiny"),
         ("spin", "hot", "spin"), ("heavy", "hot", "heavy"), ("heavy+cold", "cold", "heavy")]
res = {name: [] for name, _, _ in cases}
for _ in range(3):
    for name, which, other in cases:
        res[name].append(run(which, other, name))
fl = 2.0 * M * N * K * B
line = " | ".join(f"{k} {sorted(v)[1]:.1f}" for k, v in res.items())
print(f"GEMM [{M},{N},{K},x{B}] launch span us (in-kernel stamps, median): {line}  "
      f"(alone = {fl / sorted(res['alone'])[1] / 1e6:.0f} TF/s)", flush=True)
for k, v in phases.items():
    print(f"   {k:11s} block life {v[0]:6.2f} us = prologue {v[1]:5.2f} + first tile {v[2]:5.2f} + "
          f"K-loop {v[3]:6.2f} + epilogue {v[4]:5.2f}", flush=True)

