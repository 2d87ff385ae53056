"""GPU parity: HIP matching kernels vs the CPU oracle, through the C ABI.

Bar: bit-exact (p, converged, match indices, valid masks) on identical inputs."""
import numpy as np
import pytest
import torch

from monst3r_slam_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("b,h,w", [(1, 384, 512), (2, 384, 512), (1, 224, 224), (2, 24, 40)])
def test_iter_proj_bit_exact(oracle, dev, b, h, w):
    import mast3r_slam_backends as mb
    X11, X21, _, _ = syn.pointmap_pair_batch(b, h, w, seed=b * 7 + h)
    rwg, pts, p_init = oracle.prep_for_iter_proj(X11, X21)
    # perturb the init so the LM iterations do real work
    rng = np.random.default_rng(1)
    p_init = (p_init + rng.uniform(-3, 3, p_init.shape)).astype(np.float32)
    p_ref, c_ref = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6)
    p_gpu, c_gpu = mb.iter_proj(_t(rwg, dev), _t(pts, dev), _t(p_init, dev), 10, 1e-8, 1e-6)
    np.testing.assert_array_equal(p_gpu.cpu().numpy(), p_ref)
    np.testing.assert_array_equal(c_gpu.cpu().numpy(), c_ref)


def test_iter_proj_ragged_tail(oracle, dev):
    # n % 16 != 0 (the reference would read out of bounds; ours must be exact)
    import mast3r_slam_backends as mb
    X11, X21, _, _ = syn.pointmap_pair_batch(1, 30, 41, seed=5)
    rwg, pts, p_init = oracle.prep_for_iter_proj(X11, X21)
    n = 30 * 41 - 7
    pts, p_init = pts[:, :n].copy(), p_init[:, :n].copy()
    p_ref, c_ref = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6)
    p_gpu, c_gpu = mb.iter_proj(_t(rwg, dev), _t(pts, dev), _t(p_init, dev), 10, 1e-8, 1e-6)
    np.testing.assert_array_equal(p_gpu.cpu().numpy(), p_ref)
    np.testing.assert_array_equal(c_gpu.cpu().numpy(), c_ref)


@pytest.mark.parametrize("b,h,w", [(1, 384, 512), (2, 224, 224), (1, 30, 41)])
def test_iter_proj_fma_bit_exact_to_contracted_model(oracle, dev, b, h, w):
    """m3s_iter_proj_fma (opt-in) vs the oracle's FMA-contracted model (ref_iter_proj_fma):
    bit-exact p and converged; and end to end through match_iterative_proj with
    cfg["iter_proj_fma"]: indices and valid masks equal the oracle's contracted match."""
    from monst3r_slam_amd import _lib
    from monst3r_slam_amd import matching as M
    from monst3r_slam_amd.config import config
    X11, X21, D11, D21 = syn.pointmap_pair_batch(b, h, w, seed=b * 7 + h)
    rwg, pts, p_init = oracle.prep_for_iter_proj(X11, X21)
    rng = np.random.default_rng(1)
    p_init = (p_init + rng.uniform(-3, 3, p_init.shape)).astype(np.float32)
    n = h * w
    p_ref, c_ref = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6, contract=True)
    p = torch.empty((b, n, 2), dtype=torch.float32, device=dev)
    conv = torch.empty((b, n), dtype=torch.uint8, device=dev)
    rt, pt, pit = _t(rwg, dev), _t(pts, dev), _t(p_init, dev)
    _lib.check(_lib.load().m3s_iter_proj_fma(_lib.ptr(rt), _lib.ptr(pt), _lib.ptr(pit),
                                             _lib.ptr(p), _lib.ptr(conv), b, h, w, n, 10, 1e-8,
                                             1e-6, _lib.stream(dev)), "iter_proj_fma")
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref)
    np.testing.assert_array_equal(conv.cpu().numpy().astype(bool), c_ref)
    cfg = dict(config["matching"], iter_proj_fma=True)
    idx_ref, valid_ref = oracle.match(X11, X21, D11, D21, contract=True)
    idx, valid = M.match_iterative_proj(_t(X11, dev), _t(X21, dev), _t(D11, dev), _t(D21, dev),
                                        cfg=cfg)
    np.testing.assert_array_equal(idx.cpu().numpy(), idx_ref)
    np.testing.assert_array_equal(valid.cpu().numpy(), valid_ref)


@pytest.mark.parametrize("b,h,w", [(1, 384, 512), (2, 96, 128), (1, 31, 37)])
def test_refine_matches_bit_exact(oracle, dev, b, h, w):
    import mast3r_slam_backends as mb
    X11, X21, D11, D21 = syn.pointmap_pair_batch(b, h, w, seed=3)
    rng = np.random.default_rng(2)
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    p1 = np.stack([xx, yy], -1).reshape(1, -1, 2).repeat(b, 0)
    p1 = np.clip(p1 + rng.integers(-4, 5, p1.shape), 0, [w - 1, h - 1]).astype(np.int64)
    d11 = D11.astype(np.float16)
    d21 = D21.reshape(b, h * w, -1).astype(np.float16)
    ref = oracle.refine_matches(d11, d21, p1, 3, 5)
    (got,) = mb.refine_matches(_t(d11, dev), _t(d21, dev), _t(p1, dev), 3, 5)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


@pytest.mark.parametrize("radius,dmax", [(3, 5), (2, 3), (3, 1)])
def test_refine_matches_scattered(oracle, dev, radius, dmax):
    # scattered p1 (windows off every image edge), 24-d descriptors, 3 directions, a tile
    # count (5 x 6 = 30) that is not a multiple of the 8 XCDs: the radius-3 LDS-staged kernel
    # (every box spans the image: its global-memory path) and the generic 16x16-tile kernel
    # (radius 2) on the same inputs
    import mast3r_slam_backends as mb
    rng = np.random.default_rng(11 + radius)
    b, h, w = 3, 70, 90
    d11 = rng.normal(size=(b, h, w, 24)).astype(np.float16)
    d21 = rng.normal(size=(b, h * w, 24)).astype(np.float16)
    p1 = rng.integers(0, [w, h], size=(b, h * w, 2)).astype(np.int64)
    ref = oracle.refine_matches(d11, d21, p1, radius, dmax)
    (got,) = mb.refine_matches(_t(d11, dev), _t(d21, dev), _t(p1, dev), radius, dmax)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


@pytest.mark.parametrize("case", ["outliers", "shifted", "wide_jitter", "ties", "off_image"])
def test_refine_matches_match_fields(oracle, dev, case):
    """Radius-3 refine on match fields between the smooth and the scattered tests: smooth
    matches with 2 % scattered outliers (a tile's windows both local and spread over the
    image), a large shift (windows cut by the image edges), +-12 px jitter (a tile's
    windows wider than at +-4), descriptors on a coarse grid (many equal scores: the first
    maximum in visiting order must win, across the window columns the column-split kernel
    merges) and start points off the image (unclamped, out to +-2^40) — bit-exact against
    the oracle."""
    import mast3r_slam_backends as mb
    rng = np.random.default_rng({"outliers": 21, "shifted": 22, "wide_jitter": 23, "ties": 24,
                                 "off_image": 25}[case])
    b, h, w = 2, 96, 160
    d11 = rng.normal(size=(b, h, w, 24)).astype(np.float16)
    if case == "ties":
        d11 = (np.sign(d11) * (np.abs(d11) > 0.8)).astype(np.float16) * np.float16(0.25)
    d21 = rng.normal(size=(b, h * w, 24)).astype(np.float16)
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    p1 = np.stack([xx, yy], -1).reshape(1, -1, 2).repeat(b, 0).astype(np.int64)
    if case == "outliers":
        p1 += rng.integers(-3, 4, p1.shape)
        out = rng.uniform(size=p1.shape[:2]) < 0.02
        p1[out] = rng.integers(0, [w, h], size=(int(out.sum()), 2))
    elif case == "shifted":
        p1 += np.array([37, -21]) + rng.integers(-2, 3, p1.shape)
    elif case == "wide_jitter":
        p1 += rng.integers(-12, 13, p1.shape)
    else:
        p1 += rng.integers(-3, 4, p1.shape)
    if case == "off_image":
        p1 += rng.integers(-20, 21, p1.shape)        # up to 20 px off every edge, unclamped
        far = rng.uniform(size=p1.shape[:2]) < 0.01
        p1[far] = rng.choice([-(1 << 40), -(1 << 31), 1 << 31, 1 << 40], size=(int(far.sum()), 2))
    else:
        p1 = np.clip(p1, 0, [w - 1, h - 1])
    p1 = p1.astype(np.int64)
    ref = oracle.refine_matches(d11, d21, p1, 3, 5)
    (got,) = mb.refine_matches(_t(d11, dev), _t(d21, dev), _t(p1, dev), 3, 5)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_refine_generic_fdim(oracle, dev):
    import mast3r_slam_backends as mb
    rng = np.random.default_rng(4)
    b, h, w, f = 1, 20, 24, 17
    d11 = rng.normal(size=(b, h, w, f)).astype(np.float16)
    d21 = rng.normal(size=(b, h * w, f)).astype(np.float16)
    p1 = rng.integers(0, [w, h], size=(b, h * w, 2)).astype(np.int64)
    ref = oracle.refine_matches(d11, d21, p1, 2, 3)
    (got,) = mb.refine_matches(_t(d11, dev), _t(d21, dev), _t(p1, dev), 2, 3)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_prep_matches_golden(dev):
    import os
    from monst3r_slam_amd import matching as M
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "matching_prep.npz")))
    rwg, pts, p_init = M.prep_for_iter_proj(_t(g["X11"], dev), _t(g["X21"], dev))
    np.testing.assert_array_equal(rwg.cpu().numpy(), g["rays_with_grad"])
    np.testing.assert_array_equal(pts.cpu().numpy(), g["pts3d_norm"])
    np.testing.assert_array_equal(p_init.cpu().numpy(), g["p_init"])
    _, _, p2 = M.prep_for_iter_proj(_t(g["X11"], dev), _t(g["X21"], dev), _t(g["idx_init"], dev))
    np.testing.assert_array_equal(p2.cpu().numpy(), g["p_init_from_idx"])


@pytest.mark.parametrize("b,h,w", [(1, 384, 512), (2, 384, 512), (1, 224, 224)])
def test_match_end_to_end_bit_exact(oracle, dev, b, h, w):
    from monst3r_slam_amd import matching as M
    X11, X21, D11, D21 = syn.pointmap_pair_batch(b, h, w, seed=11)
    idx_ref, valid_ref = oracle.match(X11, X21, D11, D21)
    idx, valid = M.match(_t(X11, dev), _t(X21, dev), _t(D11, dev), _t(D21, dev))
    np.testing.assert_array_equal(idx.cpu().numpy(), idx_ref)
    np.testing.assert_array_equal(valid.cpu().numpy(), valid_ref)
    # sanity: the synthetic shift is recovered for most pixels
    assert valid_ref.mean() > 0.5


def test_match_with_init_bit_exact(oracle, dev):
    from monst3r_slam_amd import matching as M
    b, h, w = 1, 384, 512
    X11, X21, D11, D21 = syn.pointmap_pair_batch(b, h, w, seed=12)
    rng = np.random.default_rng(0)
    idx0 = np.clip(np.arange(h * w)[None] + rng.integers(-600, 600, (b, h * w)), 0,
                   h * w - 1).astype(np.int64)
    idx_ref, valid_ref = oracle.match(X11, X21, D11, D21, idx0)
    idx, valid = M.match(_t(X11, dev), _t(X21, dev), _t(D11, dev), _t(D21, dev), _t(idx0, dev))
    np.testing.assert_array_equal(idx.cpu().numpy(), idx_ref)
    np.testing.assert_array_equal(valid.cpu().numpy(), valid_ref)
