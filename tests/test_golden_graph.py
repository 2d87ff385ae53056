"""CPU: the fp32 restatement of the keyframe-graph inference (oracle/vit_ref.py
decode_symmetric_batch / inference_mono) against goldens produced by the reference's own
modules (tests/golden/make_graph_goldens.py: monst3r_utils.py:141-211 call sequence)."""
import os

import numpy as np
import pytest
import torch

from monst3r_slam_amd import weights as Wt

G = os.path.join(os.path.dirname(__file__), "golden", "graph_small.npz")


@pytest.fixture(scope="module")
def run():
    from oracle import vit_ref as V
    torch.set_flush_denormal(True)
    g = dict(np.load(G))
    am, aM = Wt.small(Wt.MONST3R), Wt.small(Wt.MAST3R)
    sdm, sdM = Wt.make_state_dict(am, 0), Wt.make_state_dict(aM, 1)
    imgs = torch.from_numpy(g["imgs"])
    H, W = imgs.shape[-2:]
    enc = [V.encode(sdm, am, imgs[k]) for k in range(imgs.shape[0])]
    pi = [int(p[0]) for p in g["pairs"]]
    pj = [int(p[1]) for p in g["pairs"]]
    fi = torch.cat([enc[i][0] for i in pi])
    fj = torch.cat([enc[j][0] for j in pj])
    posi = torch.cat([enc[i][1] for i in pi])
    posj = torch.cat([enc[j][1] for j in pj])
    X, C, D, Q = V.decode_symmetric_batch(sdm, am, sdM, aM, fi, posi, fj, posj, H, W)
    mX, mC = V.inference_mono(sdm, am, enc[0][0], enc[0][1], H, W)
    return g, dict(X=X.numpy(), C=C.numpy(), D=D.numpy(), Q=Q.numpy(), mono_X=mX.numpy(),
                   mono_C=mC.numpy())


@pytest.mark.parametrize("key", ["X", "C", "D", "Q", "mono_X", "mono_C"])
def test_graph_outputs(run, key):
    g, o = run
    assert o[key].shape == g[key].shape
    np.testing.assert_allclose(o[key], g[key], rtol=2e-4, atol=2e-5)
