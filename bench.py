"""Headline benchmark: tracking frames/sec @512x384 (+ pairwise pointmap-inference ms) on
MI355X — BASELINE.json metric, configs[1]/[2] workload.

One "step" = one tracked frame of the per-frame hot path on synthetic 384x512 input with
everything resident in HBM:
  [vit]   pair inference (MonST3R encoder of the new frame, MonST3R decoder + 2 DPT heads,
          MASt3R decoder + 2 catmlp+DPT heads; keyframe features cached) — when built
  [match] projective matching frame→keyframe (prep, iter_proj, occlusion, refine, lin)
  [track] 7-dof Sim3 ray-distance Gauss-Newton (≤50 iterations, on-device convergence)
Multi-GPU: tracking is sequential per sequence → one independent replica per rank
("replicas only"); value = frames of all ranks / max rank time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "monst3r-slam_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

H, W = 384, 512
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_DENSE_TFLOPS = 2500.0   # dense bf16 MFMA (no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


class Frame:
    """Synthetic per-frame inputs (what the ViT heads hand to matching and tracking)."""

    def __init__(self, dev, seed):
        from monst3r_slam_amd import synthetic as syn
        X11, X21, D11, D21 = syn.pair(H, W, seed=seed)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.Xkk = t(X11)[None]   # keyframe pointmap in keyframe frame (Xii)
        self.Xfk = t(X21)[None]   # frame pointmap in keyframe frame (Xji)
        self.Dk = t(D11)[None]
        self.Df = t(D21)[None]
        p = syn.tracking_problem(H, W, seed=seed)
        self.Xf = t(p["Xf"])
        self.Xk = t(p["Xk"])
        self.Qk = t(p["Qk"])
        self.valid = t(p["valid"])
        self.T_WCk = t(p["T_WCk"])
        self.T_WCf = t(p["T_WCf"])


def run_step(fr, cfg, ev=None):
    from monst3r_slam_amd import matching as M
    from monst3r_slam_amd import tracker as T
    idx, valid = M.match(fr.Xkk, fr.Xfk, fr.Dk, fr.Df, None, cfg["matching"])
    Tf, Trel, info = T.opt_pose_ray_dist_sim3(fr.Xf, fr.Xk, fr.T_WCf, fr.T_WCk, fr.Qk, fr.valid,
                                              cfg["tracking"], check=False)
    return idx, valid, Tf


def kernel_timing(fr, cfg, reps=20):
    """Average device time per launch of the matching kernels (HIP events on the stream
    the kernels run on)."""
    from monst3r_slam_amd import _lib
    from monst3r_slam_amd import matching as M
    lib = _lib.load()
    dev = fr.Xkk.device
    s = torch.cuda.current_stream(dev)
    rwg, pts, p_init = M.prep_for_iter_proj(fr.Xkk, fr.Xfk)
    n = H * W
    p = torch.empty((1, n, 2), dtype=torch.float32, device=dev)
    conv = torch.empty((1, n), dtype=torch.uint8, device=dev)
    d11 = fr.Dk.half().contiguous()
    d21 = fr.Df.reshape(1, n, -1).half().contiguous()
    p1 = (torch.stack(torch.meshgrid(torch.arange(W, device=dev), torch.arange(H, device=dev),
                                     indexing="xy"), -1).reshape(1, n, 2)).contiguous()
    p1n = torch.empty_like(p1)
    out = {}

    def timeit(fn):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        st.record(s)
        for _ in range(reps):
            fn()
        en.record(s)
        en.synchronize()
        return st.elapsed_time(en) / reps * 1e3  # us

    mc = cfg["matching"]
    out["iter_proj_us"] = timeit(lambda: lib.m3s_iter_proj(
        _lib.ptr(rwg), _lib.ptr(pts), _lib.ptr(p_init), _lib.ptr(p), _lib.ptr(conv), 1, H, W, n,
        mc["max_iter"], mc["lambda_init"], mc["convergence_thresh"], _lib.stream(dev)))
    out["refine_us"] = timeit(lambda: lib.m3s_refine_matches(
        _lib.ptr(d11), _lib.ptr(d21), _lib.ptr(p1), _lib.ptr(p1n), 1, H, W, n, 24, mc["radius"],
        mc["dilation_max"], _lib.stream(dev)))
    return out


def cpu_baseline(cfg):
    """Oracle (C port of the reference kernels + numpy tracker) on the host cores, on a
    bounded sample: one full 384x512 frame of matching + tracking."""
    from monst3r_slam_amd import synthetic as syn
    from oracle import oracle as O
    from oracle import tracker_ref as TR
    O.build()
    X11, X21, D11, D21 = syn.pair(H, W, seed=0)
    p = syn.tracking_problem(H, W, seed=0)
    t0 = time.perf_counter()
    O.match(X11[None], X21[None], D11[None], D21[None])
    TR.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"],
                              cfg["tracking"])
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": 1.0 / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": "1 frame 384x512: oracle match (C, OpenMP) + numpy tracker GN "
                      "(ViT excluded)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local_rank)
    from monst3r_slam_amd.config import default_config
    cfg = default_config()
    fr = Frame(dev, seed=rank)

    for _ in range(args.warmup):
        run_step(fr, cfg)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step(fr, cfg)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kt = kernel_timing(fr, cfg)
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        # dominant kernel: refine_matches; algorithmic bytes per launch = D11 (f16) read
        # once + D21 row + p1 in + p1 out per pixel (~25.2 MB per direction)
        n = H * W
        refine_bytes = n * 24 * 2 + n * 24 * 2 + n * 16 + n * 16
        achieved = refine_bytes / (kt["refine_us"] * 1e-6) / 1e9
        line = {
            "metric": "tracking frames/sec @512x384 + pairwise pointmap-inference ms, 1/8 MI355X",
            "value": world * args.steps / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f16",
            "data": "synthetic",
            "config": {"workload": "tracking step 384x512 (match + pose GN; ViT not yet in step)",
                       "h": H, "w": W, "parallelism": f"replicas{world}"},
            "pair_inference_ms": None,
            "stages_us": kt,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "refine_matches_kernel<24>"},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
