"""Diagnostic: HIP trunk (encoder, 4 decoders) and per-view outputs vs fp32 restatement."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import model as Mdl
from oracle import vit_ref as V
dev = torch.device("cuda:0")
small = len(sys.argv) > 1 and sys.argv[1] == "small"
m, (sdm, am, sdM, aM) = Mdl.build(dev, small=small)
sdm = {k: v.to(dev) for k, v in sdm.items()}; sdM = {k: v.to(dev) for k, v in sdM.items()}
H, W = (48, 64) if small else (384, 512)
g = torch.Generator(device=dev).manual_seed(0)
img_i = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
img_j = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
def rel(a, b):
    a = a.float(); b = b.float()
    e = (a - b).norm(dim=-1) / b.norm(dim=-1).clamp_min(1e-12)
    return f"med {e.median():.2e} p99 {e.quantile(0.99) if e.numel() < 16_000_000 else e.max():.2e} max {e.max():.2e}"
fi, pos = m.encode(img_i); fi = fi.clone()
fj, _ = m.encode(img_j); fj = fj.clone()
rfi, rpi = V.encode(sdm, am, img_i); rfj, rpj = V.encode(sdm, am, img_j)
print("enc i", rel(fi, rfi)); print("enc j", rel(fj, rfj))
gh, gw = H // 16, W // 16
hk = m.decode(fi[0], fj[0], pos, gh, gw)
# reference decoders fed with the SAME (bf16) encoder features
d1, d2 = V.decoder(sdm, am, fi.float(), rpi, fj.float(), rpj)
e1, e2 = V.decoder(sdM, aM, fi.float(), rpi, fj.float(), rpj)
for z, (a, b) in enumerate([(d1, d2), (d1, d2), (e1, e2), (e1, e2)]):
    ref = a if z % 2 == 0 else b
    print(f"z={z} h6", rel(hk["h6"][z], ref[6][0]), "| h12", rel(hk["h12"][z], ref[12][0]))
torch.backends.cuda.matmul.allow_tf32 = False
X, C, D, Q, _, _ = V.asymmetric_inference(sdm, am, sdM, aM, img_i, img_j)
out = m.pair(img_i, img_j=img_j)
for v in range(2):
    print(f"view {v} X", rel(out["X"][v], X[v]), "D", rel(out["D"][v], D[v]))
    print(f"   |X| ref med {X[v].norm(dim=-1).median():.3e} min {X[v].norm(dim=-1).min():.3e}")
