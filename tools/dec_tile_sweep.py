"""Diagnostic: every decoder GEMM of one pair (the real descriptors — epilogue flags, LN fold /
stats, RoPE, residual — recorded from decode_multi) replayed alone in a HIP graph for each
tile configuration, at the batch the step issues it (2: the per-model split chains) and at
batch 4 (one chain).  Prints us per launch and TF/s per (shape, tile).
Usage: python tools/dec_tile_sweep.py [reps]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B  # noqa: E402
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
model, _ = Mdl.build(dev)
gh, gw = B.H // 16, B.W // 16
S, E = gh * gw, 1024
g = torch.Generator(device=dev).manual_seed(3)
f1 = torch.randn(1, S, E, device=dev, generator=g).bfloat16()
f2 = torch.randn(1, S, E, device=dev, generator=g).bfloat16()
TILES = {0: "table", 1: "T128", 2: "T64", 7: "T128O2", 10: "T64D", 11: "T128D", 12: "T128W8",
         13: "T256W8", 14: "T256SQ"}


def record(split):
    model.dec_split = split
    model.ops.record = []
    model.decode_multi(f1, f2, gh, gw)
    torch.cuda.synchronize()
    rec, model.ops.record = model.ops.record, None
    seen, out = set(), []
    for d, fl, _ in rec:
        key = (d.M, d.N, d.K, d.batch, d.flags, d.mode)
        if key not in seen:
            seen.add(key)
            out.append((key, d, fl))
    return out


for split in (True, False):
    print(f"--- decoder {'split chains (batch 2)' if split else 'one chain (batch 4)'} ---",
          flush=True)
    for key, d, fl in record(split):
        row = []
        for cfg in TILES:
            dc = _lib.GemmDesc()
            ctypes.memmove(ctypes.byref(dc), ctypes.byref(d), ctypes.sizeof(d))
            if cfg:
                dc.tile_hint, dc.split_k = cfg, 1
            try:
                gr = B.capture(lambda dc=dc: [model.ops.replay_gemm(dc) for _ in range(reps)], dev)
                ms = B.time_replays(gr, dev, 5) / reps
                del gr
                row.append(f"{TILES[cfg]}={ms * 1e3:6.1f}us/{fl / ms / 1e9:5.0f}TF")
            except Exception as ex:  # noqa: BLE001
                row.append(f"{TILES[cfg]}=err")
        print(f"M{key[0]} N{key[1]} K{key[2]} b{key[3]} fl{key[4]:#x}: " + "  ".join(row),
              flush=True)
