"""Goldens for the keyframe-graph inference FROM THE REFERENCE's own network modules
(CPU, fp32, container-only): the call sequence of monst3r_utils.monst3r_decode_symmetric_batch
(:141-184) for B = 3 keyframe pairs and of monst3r_inference_mono (:187-211), on the
reduced-width models of make_vit_goldens.py (same seeded weights, strict=True).
monst3r_utils itself is not importable here (absent tp/monst3r, cv2, skimage), so its
loop body is replayed on the reference models' _encode_image / _decoder /
_downstream_head.

Writes tests/golden/graph_small.npz.  Run: python tests/golden/make_graph_goldens.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_vit_goldens import H, W, build_reference_models  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "graph_small.npz")
PAIRS = [(0, 1), (1, 2), (0, 2)]


def _dec(model, f1, p1, f2, p2, shape):
    d1, d2 = model._decoder(f1, p1, f2, p2)
    r1 = model._downstream_head(1, [t.float() for t in d1], shape)
    r2 = model._downstream_head(2, [t.float() for t in d2], shape)
    return r1, r2


@torch.no_grad()
def main():
    torch.set_flush_denormal(True)
    monst3r, mast3r = build_reference_models()
    g = torch.Generator().manual_seed(5)
    imgs = torch.rand((3, 1, 3, H, W), generator=g) * 2 - 1
    shape = torch.tensor([[H, W]], dtype=torch.int32)
    enc = [monst3r._encode_image(imgs[k], shape)[:2] for k in range(3)]
    X, C, D, Q = [], [], [], []
    for (i, j) in PAIRS:                      # monst3r_decode_symmetric_batch loop body
        (f1, p1), (f2, p2) = enc[i], enc[j]
        m11, m21 = _dec(mast3r, f1, p1, f2, p2, shape)
        m22, m12 = _dec(mast3r, f2, p2, f1, p1, shape)
        res = [m11, m21, m22, m12]
        D.append(torch.stack([r["desc"][0] for r in res]))
        Q.append(torch.stack([r["desc_conf"][0] for r in res]))
        r11, r21 = _dec(monst3r, f1, p1, f2, p2, shape)
        r22, r12 = _dec(monst3r, f2, p2, f1, p1, shape)
        res = [r11, r21, r22, r12]
        X.append(torch.stack([r["pts3d"][0] for r in res]))
        C.append(torch.stack([r["conf"][0] for r in res]))
    f, p = enc[0]                             # monst3r_inference_mono
    r11, _ = _dec(monst3r, f, p, f, p, shape)
    np.savez_compressed(
        OUT, imgs=imgs.numpy(), pairs=np.array(PAIRS), X=torch.stack(X, 1).numpy(),
        C=torch.stack(C, 1).numpy(), D=torch.stack(D, 1).numpy(), Q=torch.stack(Q, 1).numpy(),
        mono_X=r11["pts3d"].reshape(1, -1, 3).numpy(), mono_C=r11["conf"].reshape(1, -1, 1).numpy())
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
