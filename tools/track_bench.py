"""Tracker GN latency: one opt_pose_ray_dist_sim3 call at 384x512 (196,608 points) captured in
a HIP graph and replayed; convergence disabled (rel_error = delta_norm = 0) so exactly
max_iters iterations run — the slope over max_iters is the per-iteration cost, the intercept
the init / finish launches.  Optional env sweeps (M3S_TRACK_BLOCKS, M3S_TRACK_PERSISTENT) are
passed through.   python tools/track_bench.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import synthetic as syn  # noqa: E402
from monst3r_slam_amd import tracker as T  # noqa: E402
from monst3r_slam_amd.config import default_config  # noqa: E402

dev = torch.device("cuda:0")


def run(iters, reps=20):
    p = syn.tracking_problem(384, 512, seed=1)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in p.items()
         if isinstance(v, np.ndarray)}
    cfg = dict(default_config()["tracking"], max_iters=iters, rel_error=0.0, delta_norm=0.0)
    s = torch.cuda.Stream(dev)
    fn = lambda: T.opt_pose_ray_dist_sim3(t["Xf"], t["Xk"], t["T_WCf"], t["T_WCk"], t["Qk"],  # noqa
                                          t["valid"], cfg, check=False)
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            g.replay()
        e1.record(s)
        e1.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def stamps():
    """Phase timeline of workgroup 0 (debug library, make -C monst3r-slam_amd/csrc
    track_stamps): points pass, block partial, grid barrier, partial reduction, solve,
    broadcast — µs per iteration."""
    import ctypes
    from monst3r_slam_amd import _lib
    lib = ctypes.CDLL(os.path.join(ROOT, "monst3r-slam_amd/csrc/build/libm3s_track_stamps.so"))
    real = _lib.load()
    fn = lib.m3s_track_rays
    fn.restype = ctypes.c_int
    fn.argtypes = real.m3s_track_rays.argtypes
    lib.m3s_debug_track_stamps.argtypes = [ctypes.c_void_p]

    class Shim:  # route tracker.py's m3s_track_rays call into the debug library
        def __getattr__(self, k):
            return fn if k == "m3s_track_rays" else getattr(real, k)
    _lib.load = lambda: Shim()
    for _ in range(3):
        run(5, reps=1)
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 64)()
    assert lib.m3s_debug_track_stamps(buf) == 0
    st = np.array(buf[:], dtype=np.float64).reshape(8, 8) / 100.0  # µs
    names = ["points", "partial", "sweep", "combine", "solve", "bcast"]
    for it in range(5):
        d = np.diff(st[it, :7])
        print(f"iteration {it}: " + " ".join(f"{n} {v:6.2f}" for n, v in zip(names, d))
              + f" | total {st[it, 6] - st[it, 0]:6.2f} us"
              + (f" | gap to next {st[it + 1, 0] - st[it, 6]:5.2f}" if it < 4 else ""))


def main():
    if "--stamps" in sys.argv:
        return stamps()
    for blocks in (os.environ.get("BLOCKS_LIST", "256,128,64,32").split(",")):
        os.environ["M3S_TRACK_BLOCKS"] = blocks
        us = [run(k) for k in (1, 2, 3, 5, 8)]
        slope = (us[-1] - us[0]) / 7.0
        print(f"blocks {blocks:>4s}: " + " ".join(f"{k}it {u:7.1f}us" for k, u in
                                                 zip((1, 2, 3, 5, 8), us))
              + f" | per iteration {slope:6.1f} us, intercept {us[0] - slope:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
