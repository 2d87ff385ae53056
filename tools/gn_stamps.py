"""Diagnostic: the backend GN at the keyframe-graph size (P = 16 keyframes, 64 pairs as 128
two-way edges, 384 x 512 points) — wall time per iteration of mast3r_slam_backends.
gauss_newton_rays, and, with the debug library (make -C monst3r-slam_amd/csrc gn_stamps),
the LDS solve's phase timeline per iteration: per-edge blocks, assembly, Cholesky,
triangular solves, retraction / convergence (µs, thread 0, s_memrealtime).
Usage: [SCATTER=1|2] python tools/gn_stamps.py   (SCATTER=1: shifted, jittered match
indices; 2: uniformly random ones)"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import mast3r_slam_backends as mb  # noqa: E402
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd import synthetic as syn  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
ITERS = 10
g = syn.keyframe_graph(P=16, h=384, w=512, seed=5, pairs=64, two_way=True)
if os.environ.get("SCATTER") == "2":  # uniformly random match indices (the bench leg's
    rng = np.random.default_rng(1)         # random-weight descriptors scatter ~90 % of them)
    g["idx"] = rng.integers(0, g["idx"].shape[1], g["idx"].shape).astype(np.int64)
elif os.environ.get("SCATTER"):  # match indices as a moving camera's: shifted, jittered
    rng = np.random.default_rng(1)
    h, w = 384, 512
    yy, xx = np.divmod(np.arange(h * w), w)
    for e in range(g["idx"].shape[0]):
        dx, dy = rng.integers(-40, 41, 2)
        u = np.clip(xx + dx + rng.integers(-3, 4, h * w), 0, w - 1)
        v = np.clip(yy + dy + rng.integers(-3, 4, h * w), 0, h - 1)
        g["idx"][e] = v * w + u
host = {k: torch.from_numpy(np.ascontiguousarray(g[k])) for k in
        ("Twc", "Xs", "Cs", "ii", "jj", "idx", "valid", "Q")}
dv = {k: v.to(dev) for k, v in host.items()}
if os.environ.get("GN_INPUTS"):  # the bench's keyframe-graph GN call (tools/gn_host_prof.py)
    dv = {k: v.to(dev) for k, v in torch.load(os.environ["GN_INPUTS"]).items()}
    dv["valid"] = dv["valid"].reshape(dv["idx"].shape[0], -1, 1)
    dv["Q"] = dv["Q"].reshape(dv["idx"].shape[0], -1, 1)
    print({k: (tuple(v.shape), str(v.dtype)) for k, v in dv.items()}, flush=True)


def run():
    Twc = dv["Twc"].clone()
    return mb.gauss_newton_rays(Twc, dv["Xs"], dv["Cs"], dv["ii"], dv["jj"], dv["idx"],
                                dv["valid"], dv["Q"], 0.003, 10.0, 0.0, 1.5, ITERS, 0.0)


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    run()
e1.record()
e1.synchronize()
print(f"product library: {e0.elapsed_time(e1) / 5:.3f} ms per solve of {ITERS} iterations "
      f"({e0.elapsed_time(e1) / 5 / ITERS * 1e3:.0f} us per iteration)", flush=True)

# debug libraries (comma-separated in M3S_GN_STAMPS_LIB: A/B builds of gn.hip)
paths = (os.environ.get("M3S_GN_STAMPS_LIB") or os.path.join(
    ROOT, "monst3r-slam_amd/csrc/build/libm3s_gn_stamps.so")).split(",")  # build/ stays here
real = _lib.load()
names = ["edge-blocks", "assembly", "cholesky", "solves", "retract"]
for dbg_path in paths:
    lib = ctypes.CDLL(dbg_path)
    fn = lib.m3s_gauss_newton_rays
    fn.restype = ctypes.c_int
    fn.argtypes = real.m3s_gauss_newton_rays.argtypes
    lib.m3s_debug_gn_stamps.argtypes = [ctypes.c_void_p]

    class Shim:  # route the backend's call into the debug library
        def __getattr__(self, k):
            return fn if k == "m3s_gauss_newton_rays" else getattr(real, k)

    _lib.load = lambda: Shim()
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    e1.synchronize()
    print(f"{os.path.basename(dbg_path)}: {e0.elapsed_time(e1) / 5 / ITERS * 1e3:.0f} us per "
          "iteration", flush=True)
    buf = (ctypes.c_longlong * 128)()
    assert lib.m3s_debug_gn_stamps(buf) == 0
    st = np.array(buf[:], dtype=np.float64).reshape(16, 8) / 100.0  # µs
    for it in range(3):
        d = np.diff(st[it, :6])
        print(f"  iteration {it}: " + " ".join(f"{n} {v:7.2f}" for n, v in zip(names, d))
              + f" | solve kernel {st[it, 5] - st[it, 0]:7.2f} us"
              + f" | to next solve {st[it + 1, 0] - st[it, 5]:7.2f}"
              + (f" | M of poses {st[it, 6] - st[it, 0]:6.2f}, first edge batch "
                 f"{st[it, 7] - st[it, 6]:6.2f}" if st[it, 7] > 0 else ""), flush=True)
