"""Diagnostic: where the host time of the backend GN goes.  Runs the bench's keyframe-graph
leg (configs[3], one step) and profiles its final ShardedFactorGraph._solve_sharded('rays')
call (a second, warm run of it) with cProfile (torch ops that synchronise show up as their own entries), then times the
same call three more times.  GN_DUMP=path saves the call's inputs (tools/gn_stamps.py).
Usage: [GN_DUMP=path] python tools/gn_host_prof.py"""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench as B  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402
from monst3r_slam_amd import parallel as P  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
model, _ = Mdl.build(dev)
orig = P.ShardedFactorGraph._solve_sharded
calls = []


def wrapped(self, mode):
    calls.append(1)             # the bench calls it once, after its timed graph steps
    if os.environ.get("GN_DUMP"):   # the call's inputs, for tools/gn_stamps.py GN_INPUTS=...
        uniq = self.get_unique_kf_idx()
        Xs, T_WCs, Cs = self.get_poses_points(uniq)
        torch.save({"Twc": T_WCs[:, 0, :].contiguous(), "Xs": Xs.contiguous(),
                    "Cs": Cs.contiguous(), "ii": torch.cat((self.ii, self.jj)),
                    "jj": torch.cat((self.jj, self.ii)),
                    "idx": torch.cat((self.idx_ii2jj, self.idx_jj2ii)),
                    "valid": torch.cat((self.valid_match_j, self.valid_match_i)),
                    "Q": torch.cat((self.Q_ii2jj, self.Q_jj2ii))}, os.environ["GN_DUMP"])
    torch.cuda.synchronize(dev)
    orig(self, mode)            # first call: kernel loading of the torch ops it uses
    torch.cuda.synchronize(dev)
    pr = cProfile.Profile()
    pr.enable()
    orig(self, mode)
    torch.cuda.synchronize(dev)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    for rep in range(3):
        torch.cuda.synchronize(dev)
        import time
        t0 = time.perf_counter()
        orig(self, mode)
        torch.cuda.synchronize(dev)
        print(f"repeat {rep}: {(time.perf_counter() - t0) * 1e3:.2f} ms "
              f"({self.gn_iterations} iterations)", flush=True)


P.ShardedFactorGraph._solve_sharded = wrapped
out = B.keyframe_graph_bench(model, dev, 1, steps=1, warmup=1)
print({k: v for k, v in out.items() if k == "gn"}, flush=True)
