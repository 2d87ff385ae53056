"""CPU: pin the matching oracle (oracle/matching_ref.c) by known-answer tests, and the
half-arithmetic model against numpy's IEEE float16."""
import numpy as np
import pytest

from monst3r_slam_amd import synthetic as syn


def test_float_to_half_matches_numpy(oracle):
    rng = np.random.default_rng(0)
    vals = np.concatenate([
        rng.normal(0, 1, 20000), rng.normal(0, 1e-5, 5000), rng.normal(0, 1e4, 2000),
        np.array([0.0, -0.0, 65504.0, 65519.0, 65520.0, 1e-8, 6.1e-5, 5.96e-8, 2.98e-8,
                  np.inf, -np.inf]),
        # exact ties at half precision (RNE)
        (np.arange(1, 2000, dtype=np.float64) + 0.5) * 2.0 ** -10,
    ]).astype(np.float32)
    L = oracle.lib()
    got = np.array([L.ref_float_to_half(float(v)) for v in vals], np.uint16)
    np.testing.assert_array_equal(got, vals.astype(np.float16).view(np.uint16))


def test_iter_proj_identity_pair_keeps_pixel(oracle):
    # X21 == X11 and p_init = identity → every query already sits on its own ray
    X11, _, _, _ = syn.pair(48, 64, seed=1)
    X = X11[None]
    rwg, pts, p_init = oracle.prep_for_iter_proj(X, X)
    p, conv = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6)
    inner = np.zeros((48, 64), bool)
    inner[1:-1, 1:-1] = True
    inner = inner.reshape(-1)
    np.testing.assert_allclose(p[0, inner], p_init[0, inner], atol=1e-3)
    assert conv[0, inner].mean() > 0.99


def test_iter_proj_recovers_subpixel_shift(oracle):
    sx, sy = 1.5, -0.75
    X11, X21, _, _ = syn.pair(96, 128, seed=2, shift_px=(sx, sy), noise=0.0)
    rwg, pts, p_init = oracle.prep_for_iter_proj(X11[None], X21[None])
    p, conv = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6)
    yy, xx = np.meshgrid(np.arange(96), np.arange(128), indexing="ij")
    inner = ((xx > 4) & (xx < 120) & (yy > 4) & (yy < 90)).reshape(-1)
    exp = np.stack([xx + sx, yy + sy], -1).reshape(-1, 2)
    err = np.abs(p[0, inner] - exp[inner])
    assert np.median(err) < 0.05
    assert conv[0, inner].mean() > 0.9


def test_refine_one_hot_descriptors(oracle):
    # one-hot descriptors: the only positive score in the window is the true pixel
    h, w, f = 40, 48, 24
    rng = np.random.default_rng(3)
    lab = rng.integers(0, f, size=(h, w))
    D11 = np.eye(f, dtype=np.float16)[lab][None]
    # query n's descriptor = one-hot of label at (u+2, v-1) — inside the radius-3 window
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    tu = np.clip(xx + 2, 0, w - 1)
    tv = np.clip(yy - 1, 0, h - 1)
    D21 = np.eye(f, dtype=np.float16)[lab[tv, tu]].reshape(1, h * w, f)
    p1 = np.stack([xx, yy], -1).reshape(1, -1, 2).astype(np.int64)
    out = oracle.refine_matches(D11, D21, p1, 3, 1)
    # the chosen pixel must carry the query's label (score 1 > 0)
    got_lab = lab[out[0, :, 1], out[0, :, 0]]
    np.testing.assert_array_equal(got_lab, lab[tv, tu].reshape(-1))


def test_refine_zero_scores_keep_initial_pixel(oracle):
    # all candidate scores <= +0 (initial max, value-initialised c10::Half) → no move
    h, w, f = 16, 16, 24
    D11 = np.zeros((1, h, w, f), np.float16)
    D11[..., 0] = 1
    D21 = np.zeros((1, h * w, f), np.float16)
    D21[..., 0] = -1
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    p1 = np.stack([xx, yy], -1).reshape(1, -1, 2).astype(np.int64)
    out = oracle.refine_matches(D11, D21, p1, 3, 5)
    np.testing.assert_array_equal(out, p1)


def test_refine_tie_first_candidate_wins(oracle):
    # identical descriptors everywhere → strict '>' keeps the first candidate scanned
    # (u outer, v inner, dilation 5 first): (u0-15, v0-15) when inside the image
    h, w, f = 64, 64, 24
    D11 = np.full((1, h, w, f), 0.2, np.float16)
    D21 = np.full((1, h * w, f), 0.2, np.float16)
    p1 = np.array([[[32, 32]]], np.int64)
    out = oracle.refine_matches(D11, D21[:, :1], p1, 3, 5)
    # level d=5 picks (17,17); level 4 re-centred at (17,17) finds only equal scores
    np.testing.assert_array_equal(out[0, 0], [17, 17])


@pytest.mark.parametrize("flush", [False, True])
def test_refine_f16c_path_equals_software_half(oracle, monkeypatch, flush):
    """The oracle's AVX2/F16C refine (hardware RNE conversions, 8 candidate chains side by
    side) returns the same matches as the bit-level software Half arithmetic, including
    scores in the half-subnormal range and with the FTZ/DAZ mode torch.set_flush_denormal
    sets."""
    import torch
    rng = np.random.default_rng(5)
    b, h, w = 2, 24, 40
    D11 = rng.normal(size=(b, h, w, 24)).astype(np.float32)
    D21 = rng.normal(size=(b, h * w, 24)).astype(np.float32)
    D11[0] *= 3e-3                      # products ~1e-5: subnormal half partial sums
    D11[1, :, :8] = (np.sign(D11[1, :, :8]) * 6e-8)
    D11, D21 = D11.astype(np.float16), D21.astype(np.float16)
    p1 = np.stack([rng.integers(0, w, size=(b, h * w)), rng.integers(0, h, size=(b, h * w))], -1)
    prev = torch.set_flush_denormal(flush)
    try:
        monkeypatch.setenv("ORACLE_SOFT_HALF", "1")
        soft = oracle.refine_matches(D11, D21, p1, 3, 5)
        monkeypatch.setenv("ORACLE_SOFT_HALF", "0")
        fast = oracle.refine_matches(D11, D21, p1, 3, 5)
    finally:
        torch.set_flush_denormal(False)
    del prev
    assert np.array_equal(soft, fast)
    X11, X21, E11, E21 = syn.pair(48, 64, seed=3)
    p = np.stack([rng.integers(0, 64, size=(1, 48 * 64)), rng.integers(0, 48, size=(1, 48 * 64))], -1)
    monkeypatch.setenv("ORACLE_SOFT_HALF", "1")
    soft = oracle.refine_matches(E11[None].astype(np.float16), E21.reshape(1, -1, 24), p, 3, 5)
    monkeypatch.setenv("ORACLE_SOFT_HALF", "0")
    fast = oracle.refine_matches(E11[None].astype(np.float16), E21.reshape(1, -1, 24), p, 3, 5)
    assert np.array_equal(soft, fast)


def test_iter_proj_contracted_model(oracle):
    """The FMA-contracted model (ref_iter_proj_fma): the same known
    answers as the literal model (sub-pixel shift recovered, identity kept), and on the
    C3-sized 384x512 field of test_match_end_to_end_bit_exact the two models' final match
    indices differ for a few percent of the pixels (DESIGN §2 records the counts: p 105,539,
    converged 1, idx 10,122, valid 1 of 196,608)."""
    sx, sy = 1.5, -0.75
    X11, X21, _, _ = syn.pair(96, 128, seed=2, shift_px=(sx, sy), noise=0.0)
    rwg, pts, p_init = oracle.prep_for_iter_proj(X11[None], X21[None])
    p, conv = oracle.iter_proj(rwg, pts, p_init, 10, 1e-8, 1e-6, contract=True)
    yy, xx = np.meshgrid(np.arange(96), np.arange(128), indexing="ij")
    inner = ((xx > 4) & (xx < 120) & (yy > 4) & (yy < 90)).reshape(-1)
    exp = np.stack([xx + sx, yy + sy], -1).reshape(-1, 2)
    assert np.median(np.abs(p[0, inner] - exp[inner])) < 0.05
    assert conv[0, inner].mean() > 0.9
    X11, X21, D11, D21 = syn.pointmap_pair_batch(1, 384, 512, seed=11)
    i0, v0, p0, c0 = oracle.match(X11, X21, D11, D21, stages=True)
    i1, v1, p1, c1 = oracle.match(X11, X21, D11, D21, contract=True, stages=True)
    n = 384 * 512
    dp = int((p0 != p1).any(-1).sum())
    di = int((i0 != i1).sum())
    assert 0.2 * n < dp < 0.8 * n, dp          # the low bits of p move for most pixels
    assert 0 < di < 0.1 * n, di                 # truncation + refine: a few percent of idx
    assert int((v0 != v1).sum()) < 0.001 * n
