"""Diagnostic (not a bench line): which chain bounds the pipelined C3 tracking step.
Times the captured 200-frame loop with parts of the per-frame work removed by monkeypatch —
the next frame's encoder, the MASt3R DPT heads (side chain), the MonST3R DPT heads — so the
difference to the full step says how much of each chain is exposed.  Results of ablated
runs are meaningless; only their step times are read.
Usage: python tools/step_ablation.py [steps]"""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B
from monst3r_slam_amd import sequence as S
from monst3r_slam_amd.frontend import FramePipeline

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
model, tr, seq = B.setup(dev, 0, 201)
model.serial = True
tr.split_heads = True
orig_encode, orig_dpt = model.encode, model._dpt


def run(name, prefetch=True, split=True, no_enc=False, no_m3_heads=False, no_main_heads=False):
    model.encode = orig_encode

    def dpt(hooks, gh, gw, H, W, Z, wbase, wm, tag, pts, conf):
        if (tag == "mast3r" and no_m3_heads) or (tag is None and no_main_heads):
            return
        return orig_dpt(hooks, gh, gw, H, W, Z, wbase, wm, tag, pts, conf)
    model._dpt = dpt
    tr.split_heads = split
    pipe = FramePipeline(tr, (B.H, B.W)) if prefetch else None
    loop = S.SequenceLoop(tr, seq, pipe)
    loop.reset(parity=0)
    for w in range(3):
        loop.step(w)
    torch.cuda.synchronize(dev)
    if no_enc:  # captured graphs without the prefetched encoder
        model.encode = lambda img, out=None: (out, None) if out is not None else orig_encode(img)
    graphs = [B.capture(lambda: loop.step(0), dev), B.capture(lambda: loop.step(1), dev)]
    best = 1e9
    for _ in range(2):
        el = B.run_sequence(loop, graphs, steps, dev, 1)
        best = min(best, el / steps * 1e3)
    print(f"{name:40s} {best:6.3f} ms/step  {1e3 / best:6.1f} frames/s", flush=True)
    del graphs
    torch.cuda.synchronize(dev)


run("no encoder", no_enc=True)
run("no MASt3R DPT heads", no_m3_heads=True)
run("no encoder, no MASt3R DPT heads", no_enc=True, no_m3_heads=True)
run("no encoder, no DPT heads at all", no_enc=True, no_m3_heads=True, no_main_heads=True)
