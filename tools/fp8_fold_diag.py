"""fp8 LayerNorm fold vs the separate e4m3 LayerNorm launches (round 6 diagnostic): the
encoder features and the decoder hooks of one 512x512 pair, fold on / off, against each
other and against the bf16 path (cosine / relative error per tensor)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

from monst3r_slam_amd import model as Mdl  # noqa: E402


def cmp(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (f"cos {float(torch.nn.functional.cosine_similarity(a, b, dim=0)):.5f} "
            f"rel {float((a - b).norm() / b.norm()):.4f}")


dev = torch.device("cuda:0")
m, _ = Mdl.build(dev, small=len(sys.argv) > 1 and sys.argv[1] == "small")
g = torch.Generator(device=dev).manual_seed(3)
H = W = 512
img = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
img2 = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
gh, gw = H // 16, W // 16
res = {}
for mode in ("bf16", "fold", "plain"):
    m.set_fp8(mode != "bf16")
    m.fp8_fold = mode == "fold"
    f1, pos = m.encode(img)
    f1 = f1.clone()
    f2 = m.encode(img2)[0].clone()
    hooks = m.decode(f1[0], f2[0], pos, gh, gw)
    torch.cuda.synchronize()
    res[mode] = dict(feat=f1, **{k: v.clone() for k, v in hooks.items()})
m.set_fp8(False)
for k in res["bf16"]:
    print(k, "fold~bf16", cmp(res["fold"][k], res["bf16"][k]), "| plain~bf16",
          cmp(res["plain"][k], res["bf16"][k]), "| fold~plain", cmp(res["fold"][k], res["plain"][k]))
W_ = m.w
for i in (0, 1, 12, 23):
    print("enc", i, {k: float(v[i].abs().max()) if v.dim() > 0 else 0 for k, v in W_.fp8_fold_enc.items()
                     if k in ("s1", "qs1", "s2", "qs2", "qkv_c3")})
