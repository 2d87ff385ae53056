"""Diagnostic: per-stage comparison of the HIP DPT heads vs the fp32 torch restatement on
identical hook tokens (small model)."""
import os, sys
import numpy as np
import torch
import torch.nn.functional as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import model as Mdl
from oracle import vit_ref as V

dev = torch.device("cuda:0")
H, W = int(sys.argv[1]) if len(sys.argv) > 1 else 48, int(sys.argv[2]) if len(sys.argv) > 2 else 64
m, (sdm, am, sdM, aM) = Mdl.build(dev, small=True)
sd = {k: v.to(dev) for k, v in sdm.items()}
g = torch.Generator(device=dev).manual_seed(0)
img_i = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
img_j = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
out = m.pair(img_i, img_j=img_j)
torch.cuda.synchronize()
b = m._bufs
gh, gw = H // 16, W // 16
# hooks as used by HIP (z=0 → MonST3R head1)
hooks = {0: b["h0"][0:1].float()}
# rebuild the h6/h9 from decode's return: recompute via a second decode call
hk = m.decode(out["feat_i"][0], m.encode(img_j)[0][0].clone(), m.positions(1, gh, gw), gh, gw)
toks = [None] * 13
toks[0] = hk["h0"][0:1].float(); toks[6] = hk["h6"][0:1].float(); toks[9] = hk["h9"][0:1].float(); toks[12] = hk["h12"][0:1].float()
m.heads(hk, gh, gw, H, W); torch.cuda.synchronize()
# torch DPT on the same tokens, capturing intermediates
p = "downstream_head1.dpt."
ap = p + "act_postprocess."
layers = [toks[h].transpose(1, 2).reshape(1, -1, gh, gw) for h in am.hooks]
def conv(x, name, stride=1, padding=0):
    return F.conv2d(x, sd[name + ".weight"], sd.get(name + ".bias"), stride=stride, padding=padding)
l0 = F.conv_transpose2d(conv(layers[0], ap + "0.0"), sd[ap + "0.1.weight"], sd[ap + "0.1.bias"], stride=4)
l1 = F.conv_transpose2d(conv(layers[1], ap + "1.0"), sd[ap + "1.1.weight"], sd[ap + "1.1.bias"], stride=2)
l2 = conv(layers[2], ap + "2.0")
l3 = conv(conv(layers[3], ap + "3.0"), ap + "3.1", stride=2, padding=1)
def cmp(name, hip, ref):
    hip = hip.float(); ref = ref.float()
    err = (hip - ref).abs()
    idx = np.unravel_index(int(err.argmax()), tuple(err.shape))
    print(f"{name:10s} shape {tuple(ref.shape)} maxabs {err.max():.3e} at {idx} refscale {ref.abs().mean():.3e} rel {float(err.max()/ref.abs().max()):.3e}")
nhwc = lambda t: t.permute(0, 2, 3, 1)
cmp("L0", b["ap_L0"][0:1], nhwc(l0)); cmp("L1", b["ap_L1"][0:1], nhwc(l1)); cmp("L2", b["ap_L2"][0:1], nhwc(l2)); cmp("L3", b["ap_L3"][0:1], nhwc(l3))
ls = [conv(l, p + f"scratch.layer{k+1}_rn", padding=1) for k, l in enumerate([l0, l1, l2, l3])]
for k in range(4): cmp(f"rn{k}", b[f"rn{k}"][0:1], nhwc(ls[k]))
s = p + "scratch."
p4 = V._fusion(sd, s + "refinenet4", ls[3])[:, :, :ls[2].shape[2], :ls[2].shape[3]]
cmp("path4", b["path4"][0:1], nhwc(p4))
p3 = V._fusion(sd, s + "refinenet3", p4, ls[2]); cmp("path3", b["path3"][0:1], nhwc(p3))
p2 = V._fusion(sd, s + "refinenet2", p3, ls[1]); cmp("path2", b["path2"][0:1], nhwc(p2))
p1 = V._fusion(sd, s + "refinenet1", p2, ls[0]); cmp("path1", b["path1"][0:1], nhwc(p1))
h0 = conv(p1, p + "head.0", padding=1); cmp("head0", b["head0"][0:1], nhwc(h0))
hu = F.interpolate(h0, scale_factor=2, mode="bilinear", align_corners=True); cmp("head_up", b["head_up"][0:1], nhwc(hu))
h2 = F.relu(conv(hu, p + "head.2", padding=1)); cmp("head2", b["head2"][0:1], nhwc(h2))
o4 = conv(h2, p + "head.4"); fm = o4.permute(0, 2, 3, 1)
X = V.reg_dense_depth(fm[..., :3]); cmp("pts3d", b["pts3d"][0:1], X)
