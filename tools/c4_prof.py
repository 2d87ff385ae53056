"""Run only bench.py's configs[3] leg (keyframe graph: symmetric re-inference + matching +
GN over the retrieval-built graph), for rocprofv3 / A-B timing.
Usage: python tools/c4_prof.py [steps]   (M3S_SYM_CHUNK=n: pairs per symmetric chunk)"""
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
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
if os.environ.get("M3S_SYM_CHUNK"):        # A/B: most pairs per symmetric() launch set
    m.sym_chunk = int(os.environ["M3S_SYM_CHUNK"])
r = bench.keyframe_graph_bench(m, dev, 1, steps)
print(json.dumps({k: r[k] for k in ("pairs", "keyframes", "pairs_per_s", "ms_per_graph",
                                    "tflops_achieved", "gn", "valid_match_frac")}), flush=True)
