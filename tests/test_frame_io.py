"""CPU: frame preprocessing restatement (monst3r_slam_amd.monst3r_utils.resize_img /
img_norm, monst3r_utils.py:739-782, d3r/utils/image.py:23) — known answers: the output
sizes the reference's arithmetic gives, ImgNorm's range, and the crop geometry."""
import numpy as np
import pytest


@pytest.mark.parametrize("hw,size,out", [((480, 640), 512, (384, 512)),
                                         ((1024, 1024), 512, (384, 512)),   # square → 4:3
                                         ((720, 1280), 512, (288, 512)),
                                         ((480, 640), 224, (224, 224)),
                                         ((300, 200), 224, (224, 224))])
def test_resize_img_shapes(hw, size, out):
    from monst3r_slam_amd.monst3r_utils import resize_img
    img = np.random.default_rng(0).random((*hw, 3)).astype(np.float32)
    r = resize_img(img, size)
    assert r["img"].shape == (1, 3, *out)
    assert tuple(r["true_shape"][0]) == out and r["true_shape"].dtype == np.int32
    assert r["unnormalized_img"].shape == (*out, 3)
    assert -1.0 <= float(r["img"].min()) and float(r["img"].max()) <= 1.0


def test_img_norm_is_unnormalized_affine():
    from monst3r_slam_amd.monst3r_utils import resize_img
    img = np.random.default_rng(1).random((384, 512, 3)).astype(np.float32)
    r = resize_img(img, 512)                         # no resampling at the target size
    u = r["unnormalized_img"].astype(np.float32) / 255.0
    np.testing.assert_allclose(r["img"][0].numpy().transpose(1, 2, 0), (u - 0.5) / 0.5,
                               atol=1e-6)
    np.testing.assert_array_equal(r["unnormalized_img"], np.uint8(img * 255))


def test_square_ok_keeps_square():
    from monst3r_slam_amd.monst3r_utils import resize_img
    img = np.zeros((600, 600, 3), np.float32)
    assert resize_img(img, 512, square_ok=True)["img"].shape == (1, 3, 512, 512)


def test_sim3_relative_matrix_matches_lietorch_composition():
    """T_ji = T_WC_j^-1 T_WC_i as a scaled-rotation matrix + translation (the
    lietorch .matrix() of monst3r_utils.py:574-578), against the numpy Sim3 algebra."""
    import numpy as np
    import torch
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import synthetic as syn
    Ti = np.array([0.3, -0.2, 0.5, *syn.quat_from_axis_angle([1, 2, 3], 0.4), 1.3], np.float32)
    Tj = np.array([-0.1, 0.4, 0.2, *syn.quat_from_axis_angle([0, 1, -1], -0.7), 0.8], np.float32)
    sR, t = U.sim3_relative_matrix(torch.from_numpy(Ti), torch.from_numpy(Tj))
    Tji = syn.sim3_mul(syn.sim3_inv(Tj), Ti)
    X = np.random.default_rng(0).normal(size=(50, 3)).astype(np.float32)
    ref = syn.sim3_act(Tji, X)
    got = X @ sR.numpy().T + t.numpy()
    assert np.allclose(got, ref, atol=1e-5)
