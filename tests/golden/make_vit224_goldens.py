"""configs[0] golden: the FULL-WIDTH pair inference at 224x224 FROM THE REFERENCE's own network
code (CPU, fp32) — SURVEY §7.1 / §8c "224² full-width reference checksum".

Container-only (needs /root/reference).  Same procedure as make_vit_goldens.py (reference
AsymmetricCroCo3DStereo 'dpt' + AsymmetricMASt3R 'catmlp+dpt' built from the reference
checkout, seeded weights of monst3r_slam_amd.weights.make_state_dict loaded strict, the call
sequence of monst3r_utils.monst3r_asymmetric_inference :255-297), but at the production
widths (ViT-L encoder 1024, ViT-B decoder 768) and seeds of model.build (0 / 1), on a
224x224 pair.  To keep the fixture small: X, C, Q and the encoder features stored as f16
(the tests compare at bf16-network tolerances, f16 storage error is ~5e-4 relative), the
24-d descriptors on every 7th pixel of every 7th row, plus f64 checksums of the full tensors.

Writes tests/golden/vit224_full.npz.  Run:  python tests/golden/make_vit224_goldens.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_vit_goldens as base  # noqa: E402

OUT = os.path.join(HERE, "vit224_full.npz")
S = 224


def build_full():
    from monst3r_slam_amd import weights as Wt
    small = Wt.small
    Wt.small = lambda a: a             # production widths through the same builder
    try:
        return base.build_reference_models()
    finally:
        Wt.small = small


@torch.no_grad()
def main():
    torch.set_flush_denormal(True)
    torch.set_num_threads(os.cpu_count() or 8)
    monst3r, mast3r = build_full()
    g = torch.Generator().manual_seed(base.SEED_IMG)
    img_i = torch.rand((1, 3, S, S), generator=g) * 2 - 1
    img_j = torch.rand((1, 3, S, S), generator=g) * 2 - 1
    shape = torch.tensor([[S, S]], dtype=torch.int32)
    fi, pi, _ = monst3r._encode_image(img_i, shape)
    fj, pj, _ = monst3r._encode_image(img_j, shape)
    d1, d2 = monst3r._decoder(fi, pi, fj, pj)
    r11 = monst3r._downstream_head(1, [t.float() for t in d1], shape)
    r21 = monst3r._downstream_head(2, [t.float() for t in d2], shape)
    e1, e2 = mast3r._decoder(fi, pi, fj, pj)
    m11 = mast3r._downstream_head(1, [t.float() for t in e1], shape)
    m21 = mast3r._downstream_head(2, [t.float() for t in e2], shape)
    X = torch.stack([r11["pts3d"][0], r21["pts3d"][0]])
    C = torch.stack([r11["conf"][0], r21["conf"][0]])
    D = torch.stack([m11["desc"][0], m21["desc"][0]])
    Q = torch.stack([m11["desc_conf"][0], m21["desc_conf"][0]])
    sums = {f"sum_{k}": np.array([float(v.double().sum()), float(v.double().abs().sum())])
            for k, v in dict(X=X, C=C, D=D, Q=Q, feat_i=fi, feat_j=fj).items()}
    np.savez_compressed(
        OUT, img_i=img_i.numpy(), img_j=img_j.numpy(), feat_i=fi.half().numpy(),
        feat_j=fj.half().numpy(), X=X.half().numpy(), C=C.half().numpy(), Q=Q.half().numpy(),
        D_sub=D[:, ::7, ::7].numpy(), **sums)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
