"""Per-shape GEMM time of one pair inference, measured the way bench.gemm_replay does: the
pair's launches are recorded (descriptors, same buffers) during an eager run, then each
shape class is replayed back-to-back in its own HIP graph and timed with HIP events
(eager per-launch events are host-bound: the ctypes wrapper costs more than a short GEMM).
Optional M3S_GEMM_TILE / SPLIT overrides apply to the replayed descriptors."""
import collections
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
img = torch.rand(1, 3, 384, 512, device=dev) * 2 - 1
feat, _ = m.encode(img)
feat = feat.clone()
m.ops.record = []
m.pair(img, feat_j=feat)
torch.cuda.synchronize()
rec, m.ops.record = m.ops.record, None
groups = collections.OrderedDict()
for d, fl, _f8 in rec:
    key = (d.M, d.N, d.K, d.batch, "conv" if d.mode == 1 else "gemm", d.flags)
    groups.setdefault(key, []).append((d, fl))
tot_ms = 0.0
rows = []
for key, lst in groups.items():
    reps = max(1, 40 // len(lst))
    g = bench.capture(lambda lst=lst: [m.ops.replay_gemm(d) for d, _ in lst * reps], dev)
    ms = bench.time_replays(g, dev, 5) / reps
    del g
    fl = sum(f for _, f in lst)
    tot_ms += ms
    rows.append((ms, key, len(lst), fl))
print(f"total gemm ms {tot_ms:.3f} launches {len(rec)} "
      f"({sum(r[3] for r in rows) / tot_ms / 1e9:.0f} TF/s)")
for ms, key, n, fl in sorted(rows, key=lambda r: -r[0]):
    print(f"{str(key):52s} n={n:3d} ms={ms:7.3f} ({100 * ms / tot_ms:4.1f}%) "
          f"us/launch={ms / n * 1e3:7.1f} TF/s={fl / (ms * 1e-3) / 1e12:7.1f}", flush=True)
