"""Generate ViT/DPT golden fixtures FROM THE REFERENCE's own network code (CPU, fp32).

Container-only (needs /root/reference; never run on the GPU box).  Builds the reference
AsymmetricCroCo3DStereo (MonST3R arch, head 'dpt') and AsymmetricMASt3R (head
'catmlp+dpt') from /root/reference/MASt3R-SLAM/thirdparty/mast3r at reduced width
(same topology; monst3r_slam_amd.weights.small), loads the seeded weights of
monst3r_slam_amd.weights.make_state_dict with strict=True, and replays the call sequence
of monst3r_utils.monst3r_asymmetric_inference (:255-297) — that module itself is not
importable here (it imports the absent tp/monst3r submodule, cv2 and skimage).
The reference uses its pure-PyTorch RoPE2D fallback (curope is CUDA-only).

Writes tests/golden/vit_small.npz.  Run: python tests/golden/make_vit_goldens.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "monst3r-slam_amd"))
sys.path.insert(0, "/root/reference/MASt3R-SLAM/thirdparty/mast3r")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vit_small.npz")
H, W = 48, 64
SEED_MONST3R, SEED_MAST3R, SEED_IMG = 0, 1, 2


def build_reference_models():
    import mast3r.utils.path_to_dust3r  # noqa: F401
    from dust3r.model import AsymmetricCroCo3DStereo
    from mast3r.model import AsymmetricMASt3R
    from monst3r_slam_amd import weights as Wt
    inf = float("inf")
    am, aM = Wt.small(Wt.MONST3R), Wt.small(Wt.MAST3R)
    monst3r = AsymmetricCroCo3DStereo(
        pos_embed="RoPE100", patch_embed_cls="PatchEmbedDust3R", img_size=(512, 512),
        head_type="dpt", output_mode="pts3d", depth_mode=("exp", -inf, inf),
        conf_mode=("exp", 1, inf), enc_embed_dim=am.enc_dim, enc_depth=am.enc_depth,
        enc_num_heads=am.enc_heads, dec_embed_dim=am.dec_dim, dec_depth=am.dec_depth,
        dec_num_heads=am.dec_heads, freeze="encoder", landscape_only=False)
    mast3r = AsymmetricMASt3R(
        enc_depth=aM.enc_depth, dec_depth=aM.dec_depth, enc_embed_dim=aM.enc_dim,
        dec_embed_dim=aM.dec_dim, enc_num_heads=aM.enc_heads, dec_num_heads=aM.dec_heads,
        pos_embed="RoPE100", img_size=(512, 512), head_type="catmlp+dpt",
        output_mode="pts3d+desc24", depth_mode=("exp", -inf, inf), conf_mode=("exp", 1, inf),
        patch_embed_cls="PatchEmbedDust3R", two_confs=True, desc_conf_mode=("exp", 0, inf),
        landscape_only=False)
    monst3r.load_state_dict(Wt.make_state_dict(am, SEED_MONST3R), strict=True)
    mast3r.load_state_dict(Wt.make_state_dict(aM, SEED_MAST3R), strict=True)
    return monst3r.eval(), mast3r.eval()


def images():
    g = torch.Generator().manual_seed(SEED_IMG)
    img_i = torch.rand((1, 3, H, W), generator=g) * 2 - 1
    img_j = torch.rand((1, 3, H, W), generator=g) * 2 - 1
    return img_i, img_j


@torch.no_grad()
def main():
    torch.set_flush_denormal(True)
    monst3r, mast3r = build_reference_models()
    img_i, img_j = images()
    shape = torch.tensor([[H, W]], dtype=torch.int32)
    fi, pi, _ = monst3r._encode_image(img_i, shape)
    fj, pj, _ = monst3r._encode_image(img_j, shape)
    d1, d2 = monst3r._decoder(fi, pi, fj, pj)
    d1, d2 = list(d1), list(d2)
    r11 = monst3r._downstream_head(1, [t.float() for t in d1], shape)
    r21 = monst3r._downstream_head(2, [t.float() for t in d2], shape)
    e1, e2 = mast3r._decoder(fi, pi, fj, pj)
    e1, e2 = list(e1), list(e2)
    m11 = mast3r._downstream_head(1, [t.float() for t in e1], shape)
    m21 = mast3r._downstream_head(2, [t.float() for t in e2], shape)
    X = torch.stack([r11["pts3d"][0], r21["pts3d"][0]])
    C = torch.stack([r11["conf"][0], r21["conf"][0]])
    D = torch.stack([m11["desc"][0], m21["desc"][0]])
    Q = torch.stack([m11["desc_conf"][0], m21["desc_conf"][0]])
    np.savez_compressed(OUT, img_i=img_i.numpy(), img_j=img_j.numpy(), feat_i=fi.numpy(),
                        feat_j=fj.numpy(), pos_i=pi.numpy(), dec1_last=d1[-1].numpy(),
                        dec2_last=d2[-1].numpy(), dec1_6=d1[6].numpy(), X=X.numpy(),
                        C=C.numpy(), D=D.numpy(), Q=Q.numpy(),
                        mast3r_pts3d=torch.stack([m11["pts3d"][0], m21["pts3d"][0]]).numpy(),
                        mast3r_conf=torch.stack([m11["conf"][0], m21["conf"][0]]).numpy())
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
