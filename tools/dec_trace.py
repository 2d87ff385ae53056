"""Diagnostic: the decoder chain alone (one chain, `problems` = 4 or 8 decoder problems),
replayed from a HIP graph, for a rocprofv3 kernel trace: per-launch device time by (kernel,
grid) and the gaps between consecutive launches (tools/dec_trace_report.py).
Usage: rocprofv3 --kernel-trace -d DIR -o dec -- python tools/dec_trace.py [problems] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

problems = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
model, _ = Mdl.build(dev)
model.dec_split = False
gh, gw = B.H // 16, B.W // 16
S, E = gh * gw, 1024
G = problems // 4
g = torch.Generator(device=dev).manual_seed(3)
f1 = torch.randn(G, S, E, device=dev, generator=g).bfloat16()
f2 = torch.randn(G, S, E, device=dev, generator=g).bfloat16()
gr = B.capture(lambda: model.decode_multi(f1, f2, gh, gw), dev)
torch.cuda.synchronize()
ms = B.time_replays(gr, dev, reps)
print(f"decoder {problems} problems: {ms * 1e3:.1f} us per replay", flush=True)
