"""Diagnostic (not a bench line): what batching two frames' pair inference buys.
Times (HIP graph replay, alone on the chip) the per-frame pair work of the C3 step —
decoders (both models) + DPT heads + local features vs the cached keyframe features — for
one frame (the current schedule: the decoder split by model on two streams, the MASt3R heads
on a side stream) against two frames batched in every launch (8 decoder problems, 8 heads).
Usage: python tools/batch_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
model, _ = Mdl.build(dev)
H, W = B.H, B.W
gh, gw = H // 16, W // 16
S, E = gh * gw, 1024
g = torch.Generator(device=dev).manual_seed(3)
f2 = torch.randn(2, S, E, device=dev, generator=g).bfloat16()
fk = torch.randn(1, S, E, device=dev, generator=g).bfloat16()
fk2 = fk.expand(2, S, E).contiguous()


def t(name, fn, reps=20):
    gr = B.capture(fn, dev)
    ms = B.time_replays(gr, dev, reps)
    print(f"{name:52s} {ms * 1e3:8.1f} us", flush=True)
    del gr
    return ms


def dec1():
    return model.decode_multi(f2[0:1], fk, gh, gw)


def dec2():
    return model.decode_multi(f2, fk2, gh, gw)


def pair1():
    hk = dec1()
    model.heads(hk, gh, gw, H, W, split=True)
    model.join()


def pair2():
    hk = dec2()
    model.heads(hk, gh, gw, H, W)


def heads1():
    model.heads(h1, gh, gw, H, W, split=True)
    model.join()


def heads2():
    model.heads(h2, gh, gw, H, W)


d1 = t("decoder, 1 frame (2 chains of 2 problems)", dec1)
d2 = t("decoder, 2 frames batched (1 chain of 8 problems)", dec2)
model.dec_split = False
d1b = t("decoder, 1 frame (1 chain of 4 problems)", dec1)
model.dec_split = True
h1 = {k: v.clone() for k, v in dec1().items()}
h2 = {k: v.clone() for k, v in dec2().items()}
torch.cuda.synchronize()
e1 = t("heads, 1 frame (MASt3R heads on a side stream)", heads1)
e2 = t("heads, 2 frames batched (8 problems)", heads2)
p1 = t("pair, 1 frame", pair1)
p2 = t("pair, 2 frames batched", pair2)
print(f"per frame: decoder {d1 * 1e3:.0f} -> {d2 / 2 * 1e3:.0f} us, heads {e1 * 1e3:.0f} -> "
      f"{e2 / 2 * 1e3:.0f} us, pair {p1 * 1e3:.0f} -> {p2 / 2 * 1e3:.0f} us", flush=True)
