"""CPU: the oracle's numpy restatement of the matching prep / glue against goldens
produced by the reference's own Python (tests/golden/make_goldens.py)."""
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(__file__), "golden", "matching_prep.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(G))


def test_prep_matches_reference(oracle, gold):
    rwg, pts, p_init = oracle.prep_for_iter_proj(gold["X11"], gold["X21"])
    # bit-exact: FMA orders pinned to the reference's torch-CPU run
    np.testing.assert_array_equal(rwg, gold["rays_with_grad"])
    np.testing.assert_array_equal(pts, gold["pts3d_norm"])
    np.testing.assert_array_equal(p_init, gold["p_init"])
    _, _, p2 = oracle.prep_for_iter_proj(gold["X11"], gold["X21"], gold["idx_init"])
    np.testing.assert_array_equal(p2, gold["p_init_from_idx"])


def test_occlusion_and_lin_match_reference(oracle, gold):
    # the reference's glue applied to fixed kernel outputs (stubbed in the generator)
    X11, X21 = gold["X11"], gold["X21"]
    b, h, w, _ = X11.shape
    p1, valid = oracle.match_occlusion(X11, X21, gold["p_stub"], gold["conv_stub"], 0.1)
    np.testing.assert_array_equal(valid[..., None], gold["valid"])
    np.testing.assert_array_equal(p1[..., 0] + w * p1[..., 1], gold["idx"])
