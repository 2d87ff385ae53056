"""Per-launch-shape summary of the step's block log (bench.py M3S_BLOCKLOG_OUT + its
--timeline-out JSON): blocks, mean block lifetime and its GEMM phases (prologue issue,
first K-tile wait, K-loop, epilogue) in us, for one replayed step.
Usage: python tools/blocklog_report.py blocklog.npz timeline.json [graph_index]"""
import json
import sys
from collections import defaultdict

import numpy as np

z = np.load(sys.argv[1])
tl = json.load(open(sys.argv[2]))
gi = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lg, sl, gr = z["log"], z["slot"], z["graphs"]
a, b = gr[gi]
sel = (sl >= a) & (sl < b)
L, S = lg[sel], sl[sel] - a
launches = tl["launches"]
agg = defaultdict(lambda: np.zeros(9))
for s in np.unique(S):
    m = S == s
    x = L[m].astype(np.float64)
    life = (x[:, 1] - x[:, 0]) * 1e-2
    ph = x[:, 4:8]
    ok = (ph > 0).all(1)
    pro = (ph[ok, 0] - x[ok, 0]) * 1e-2
    first = (ph[ok, 1] - ph[ok, 0]) * 1e-2
    loop = (ph[ok, 2] - ph[ok, 1]) * 1e-2
    epi = (x[ok, 1] - ph[ok, 2]) * 1e-2
    # epilogue split at mark 3: operand setup + accumulators → LDS + barrier, then the
    # vector pass (LDS reads, epilogue math, stores)
    e_lds = (ph[ok, 3] - ph[ok, 2]) * 1e-2
    ln = launches[s] if s < len(launches) else {"kind": "?", "dims": []}
    key = (ln["kind"], tuple(ln["dims"]), int(m.sum()))
    v = agg[key]
    v += [1, life.mean(), pro.mean() if ok.any() else 0, first.mean() if ok.any() else 0,
          loop.mean() if ok.any() else 0, epi.mean() if ok.any() else 0,
          (ln.get("gflop") or 0), 0, e_lds.mean() if ok.any() else 0]
rows = sorted(agg.items(), key=lambda kv: -kv[1][0] * kv[1][1] * kv[0][2])
print("kind  dims                          blocks  n   life  prolog first  kloop   epi (to-LDS  vec)  (us, mean per block)")
for (kind, dims, nb), v in rows:
    n = v[0]
    print(f"{kind:5s} {str(list(dims)):28s} {nb:6d} {int(n):3d} {v[1]/n:6.1f} {v[2]/n:6.2f} "
          f"{v[3]/n:6.2f} {v[4]/n:6.1f} {v[5]/n:6.2f} ({v[8]/n:5.2f} {(v[5]-v[8])/n:5.2f})")
