"""CPU: the fp32 ViT/DPT restatement (oracle/vit_ref.py) against goldens produced by the
reference's own network modules (tests/golden/make_vit_goldens.py), small-width models
with identical seeded weights."""
import os

import numpy as np
import pytest
import torch

from monst3r_slam_amd import weights as Wt

G = os.path.join(os.path.dirname(__file__), "golden", "vit_small.npz")


@pytest.fixture(scope="module")
def run():
    from oracle import vit_ref as V
    torch.set_flush_denormal(True)
    g = dict(np.load(G))
    am, aM = Wt.small(Wt.MONST3R), Wt.small(Wt.MAST3R)
    sdm = Wt.make_state_dict(am, 0)
    sdM = Wt.make_state_dict(aM, 1)
    X, C, D, Q, (fi, _), _ = V.asymmetric_inference(sdm, am, sdM, aM,
                                                    torch.from_numpy(g["img_i"]),
                                                    torch.from_numpy(g["img_j"]))
    return g, dict(X=X.numpy(), C=C.numpy(), D=D.numpy(), Q=Q.numpy(), feat_i=fi.numpy())


def test_encoder_features(run):
    g, o = run
    np.testing.assert_allclose(o["feat_i"], g["feat_i"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("key", ["X", "C", "D", "Q"])
def test_pair_outputs(run, key):
    g, o = run
    # same fp32 math, different op grouping (fused qkv split, conv algorithms): 1e-4 rel
    np.testing.assert_allclose(o[key], g[key], rtol=2e-4, atol=2e-5)
