"""Run only bench.py's configs[4] leg (fp8 512x512 dyn-mask frame), for rocprofv3.
Usage: python tools/c5_prof.py [steps] [mode,mode,...]  (modes: fp8, fp8_convs, bf16)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
if len(sys.argv) > 2:
    print(json.dumps(bench.c5_bench(m, dev, steps, tuple(sys.argv[2].split(",")))))
else:
    print(json.dumps(bench.c5_bench(m, dev, steps)))
