"""Per-launch GEMM timing of one pair inference (HIP events), grouped by shape."""
import collections, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import model as Mdl
from monst3r_slam_amd import _lib
dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
img = torch.rand(1, 3, 384, 512, device=dev) * 2 - 1
feat, _ = m.encode(img); feat = feat.clone()
orig = m.ops.gemm
rec = []
def gemm(A, B, C, M, N, K, batch=1, **kw):
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); orig(A, B, C, M, N, K, batch, **kw); e1.record(st)
    rec.append(((M, N, K, batch, "conv" if kw.get("conv") else ("convt" if kw.get("convt") else "gemm")), e0, e1))
m.ops.gemm = gemm
for it in range(3):
    rec.clear(); m.pair(img, feat_j=feat); torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for key, e0, e1 in rec:
    M, N, K, b, kind = key
    a = agg[key]; a[0] += 1; a[1] += e0.elapsed_time(e1); a[2] += 2.0 * M * N * K * b
tot = sum(a[1] for a in agg.values())
print(f"total gemm ms {tot:.3f} launches {len(rec)}")
for key, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{str(key):45s} n={n:3d} ms={ms:7.3f} ({100*ms/tot:4.1f}%) TF/s={fl/(ms*1e-3)/1e12:7.1f}")
