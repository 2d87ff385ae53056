"""GPU parity: backend GN (mast3r_slam_backends.gauss_newton_*) and the fused tracker vs
the CPU oracle.  Floating-point work with a different reduction order (f32 partial sums,
f64 solve): poses compared with an absolute tolerance stated per test."""
import numpy as np
import pytest
import torch

from monst3r_slam_amd import synthetic as syn
from monst3r_slam_amd.config import default_config

pytestmark = pytest.mark.gpu

POSE_TOL = 2e-5   # |ΔT| elementwise after the same number of GN iterations
TRACK_TOL = 1e-4  # tracker: up to 50 f32 iterations, convergence test on f32 cost


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _gn_case(g, dev):
    return [_t(g[k], dev) for k in ("Twc", "Xs", "Cs", "ii", "jj", "idx", "valid", "Q")]


@pytest.mark.parametrize("P,h,w,iters", [(5, 48, 64, 1), (5, 48, 64, 10), (8, 96, 128, 3)])
def test_gn_rays_parity(oracle, dev, P, h, w, iters):
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=P, h=h, w=w, seed=P + h)
    Twc_ref = g["Twc"].copy()
    ref = oracle.gauss_newton("rays", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                              g["valid"], g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0,
                              Q_thresh=1.5, max_iter=iters, delta_thresh=1e-8)
    Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
    (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5,
                                 iters, 1e-8)
    np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(dx.cpu().numpy(), ref["dx"], atol=POSE_TOL, rtol=0)


@pytest.mark.parametrize("P", [2, 19, 20, 21, 22, 24])
def test_gn_rays_solve_paths(oracle, dev, P):
    """The fp64 solve runs LDS-resident (system assembled by block row in edge order,
    Cholesky in LDS, one-wave triangular solves) while n = 7(P - 1) <= 140 and in global
    memory beyond: both paths — the round-5 edge (P = 19, n = 126: two row registers per
    lane), rows past 128 (P = 20, 21: a third row register in the panel factor and the
    triangular solves, the wide update's second row pass) and past the LDS capacity (P = 22,
    24) — vs the oracle's dense Cholesky."""
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=P, h=24, w=32, seed=P)
    for iters in (1, 3):
        Twc_ref = g["Twc"].copy()
        ref = oracle.gauss_newton("rays", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                                  g["valid"], g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0,
                                  Q_thresh=1.5, max_iter=iters, delta_thresh=1e-8)
        Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
        (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5,
                                     iters, 1e-8)
        dx, ref_dx = dx.cpu().numpy(), ref["dx"]
        if iters == 1:
            # the first step (|dx| up to 0.15): f32 edge sums in another order than the
            # oracle's, amplified along the 19-24 pose gauge chain — measured relative error
            # of the whole step <= 1.2e-3 (poses after it off by up to 1.2e-4)
            rel = np.linalg.norm(dx - ref_dx) / np.linalg.norm(ref_dx)
            assert rel < 5e-3, f"first step relative error {rel:.2e}"
        else:
            # converged poses: the chain's f32 noise (measured <= 3.7e-5 at P = 24 on poses of
            # magnitude ~1.2) — relative 5e-5 on top of the absolute bar.  The third step
            # itself (|dx| ~ 1e-5 at P = 2) is the rounding noise of the gradient sums.
            np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=POSE_TOL, rtol=5e-5)


@pytest.mark.parametrize("P", [2, 16, 19, 20, 21])
def test_gn_lds_solve_equals_global_solve(dev, P):
    """The LDS-resident solve (block-row assembly in edge order, look-ahead LDS Cholesky,
    one-wave triangular solves) performs the global-memory solve's operations in the same order:
    poses and steps bit-identical."""
    import mast3r_slam_backends as mb
    from monst3r_slam_amd import _lib
    g = syn.keyframe_graph(P=P, h=24, w=32, seed=100 + P)
    outs = []
    for force in (0, 1):
        _lib.load().m3s_gn_force_global_solve(force)
        try:
            Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
            (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0,
                                         1.5, 5, 1e-8)
            outs.append((Twc.cpu(), dx.cpu()))
        finally:
            _lib.load().m3s_gn_force_global_solve(0)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_gn_lds_solve_equals_global_solve_many_edges(dev):
    """Past 1,024 edges (64 per wave of the LDS solve: the per-wave pose-rank registers are
    refilled, the assembly's ballot walks 18 chunks of 64 edges) the LDS solve still performs
    the global solve's operations in the same order: 1,120 two-way edges (the 28 pairs of 8
    keyframes, each 20 times with its own validity and Q), poses and steps bit-identical."""
    import mast3r_slam_backends as mb
    from monst3r_slam_amd import _lib
    g = syn.keyframe_graph(P=8, h=8, w=16, seed=77, pairs=28, two_way=True)
    rng = np.random.default_rng(5)
    reps = 20
    g = dict(g)
    for k in ("ii", "jj", "idx"):
        g[k] = np.concatenate([g[k]] * reps)
    E, N = g["idx"].shape
    assert E == 1120
    g["valid"] = rng.uniform(size=(E, N, 1)) < 0.9
    g["Q"] = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(E, N, 1)))).astype(np.float32)
    outs = []
    for force in (0, 1):
        _lib.load().m3s_gn_force_global_solve(force)
        try:
            Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
            (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0,
                                         1.5, 3, 1e-8)
            outs.append((Twc.cpu(), dx.cpu()))
        finally:
            _lib.load().m3s_gn_force_global_solve(0)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.isfinite(outs[0][0]).all() and outs[0][1].abs().sum() > 0


def test_gn_invalid_matches_ignore_their_index(dev):
    """The edge pass packs the match index with the validity folded in (-1 where invalid,
    `gn_pack_kernel`): an invalid match's index is never read, whatever it holds — the
    reference's `valid ? idx : 0`.  Garbage indices (negative, past N) under invalid
    matches give the same poses, bit for bit, as zeros there."""
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=6, h=24, w=32, seed=31)
    outs = []
    for fill in (0, -7, 10 ** 9):
        Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
        idx = torch.where(valid[..., 0], idx, torch.full_like(idx, fill))
        (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx.contiguous(), valid, Q, 0.003,
                                     10.0, 0.0, 1.5, 4, 1e-8)
        outs.append((Twc.cpu(), dx.cpu()))
    for t, d in outs[1:]:
        assert torch.equal(t, outs[0][0]) and torch.equal(d, outs[0][1])


def test_gn_points_parity(oracle, dev):
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=4, h=48, w=64, seed=3)
    Twc_ref = g["Twc"].copy()
    oracle.gauss_newton("points", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                        g["valid"], g["Q"], sig0=0.05, C_thresh=0.0, Q_thresh=1.5, max_iter=5,
                        delta_thresh=1e-8)
    Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
    mb.gauss_newton_points(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.05, 0.0, 1.5, 5, 1e-8)
    np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=POSE_TOL, rtol=0)


def test_gn_calib_parity(oracle, dev):
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=4, h=48, w=64, seed=4)
    Twc_ref = g["Twc"].copy()
    oracle.gauss_newton("calib", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                        g["valid"], g["Q"], sig0=1.0, sig1=10.0, C_thresh=0.0, Q_thresh=1.5,
                        max_iter=3, delta_thresh=1e-8, K=g["K"], height=48, width=64,
                        pixel_border=-10, z_eps=1e-6)
    Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
    mb.gauss_newton_calib(Twc, Xs, Cs, _t(g["K"], dev), ii, jj, idx, valid, Q, 48, 64, -10, 1e-6,
                          1.0, 10.0, 0.0, 1.5, 3, 1e-8)
    # identity correspondences are not pixel-consistent under calib projection: residuals
    # of tens of pixels make this system ill-conditioned, so f32 summation-order noise is
    # amplified over 3 iterations → relative tolerance 1e-4
    np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=1e-4, rtol=1e-4)


def test_gn_global_ids_and_not_pd(oracle, dev):
    # keyframe ids are global (sparse) and all matches invalid → zero step, poses untouched
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=3, h=8, w=8, seed=2)
    Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
    ii, jj = ii * 7 + 3, jj * 7 + 3
    before = Twc.clone()
    (dx,) = mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, torch.zeros_like(valid), Q, 0.003,
                                 10.0, 0.0, 1.5, 10, 1e-8)
    assert torch.equal(Twc, before)
    assert torch.count_nonzero(dx) == 0


@pytest.mark.parametrize("extra", [1, 2])
def test_gn_more_unique_ids_than_poses_is_rejected_cleanly(oracle, dev, extra):
    """|unique(ii, jj)| > P (the reference's size check, gn_kernels.cu:1160-1170): ranks then
    reach past the P poses, so no kernel of the solve may run — the call raises, Twc is left
    untouched (no out-of-bounds pose / counter / partial access on the way), and a valid call
    on the same device afterwards still matches the oracle."""
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=4, h=24, w=32, seed=12)
    Twc, Xs, Cs, ii, jj, idx, valid, Q = _gn_case(g, dev)
    bad_ii = ii.clone()
    for t in range(extra):
        bad_ii[t] = 50 + t          # keyframe ids no pose exists for
    before = Twc.clone()
    with pytest.raises(RuntimeError, match="unique keyframes"):
        mb.gauss_newton_rays(Twc, Xs, Cs, bad_ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5, 5,
                             1e-8)
    torch.cuda.synchronize()
    assert torch.equal(Twc, before)
    Twc_ref = g["Twc"].copy()
    oracle.gauss_newton("rays", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                        g["valid"], g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0, Q_thresh=1.5,
                        max_iter=3, delta_thresh=1e-8)
    mb.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5, 3, 1e-8)
    np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=POSE_TOL, rtol=0)


@pytest.mark.parametrize("stride", [3, 70001])
def test_gn_global_ids_parity(oracle, dev, stride):
    # stride 3: ids within a 2^17 range (bitmap ranks); 70001: wider (the O(M^2) fallback)
    import mast3r_slam_backends as mb
    g = syn.keyframe_graph(P=5, h=24, w=32, seed=9)
    Twc_ref = g["Twc"].copy()
    ii_g, jj_g = g["ii"] * stride + 100, g["jj"] * stride + 100
    oracle.gauss_newton("rays", Twc_ref, g["Xs"], g["Cs"], ii_g, jj_g, g["idx"], g["valid"],
                        g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0, Q_thresh=1.5, max_iter=4,
                        delta_thresh=1e-8)
    Twc, Xs, Cs, _, _, idx, valid, Q = _gn_case(g, dev)
    mb.gauss_newton_rays(Twc, Xs, Cs, _t(ii_g, dev), _t(jj_g, dev), idx, valid, Q, 0.003, 10.0,
                         0.0, 1.5, 4, 1e-8)
    np.testing.assert_allclose(Twc.cpu().numpy(), Twc_ref, atol=POSE_TOL, rtol=0)


# launch modes of the GN: persistent (default), one launch per iteration, and the
# persistent launch forced to abort at its 2nd barrier (co-residency lost) with the
# remaining iterations run by the recovery path of the finish launch
LAUNCH_MODES = {"persistent": {}, "per_iteration": {"M3S_TRACK_PERSISTENT": "0"},
                "recovered": {"M3S_TRACK_ABORT_AT": "1"}}


def _launch_mode(monkeypatch, mode):
    for k in ("M3S_TRACK_PERSISTENT", "M3S_TRACK_ABORT_AT", "M3S_TRACK_SPIN_LIMIT"):
        monkeypatch.delenv(k, raising=False)
    for k, v in LAUNCH_MODES[mode].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("mode", list(LAUNCH_MODES))
@pytest.mark.parametrize("h,w", [(384, 512), (96, 128)])
def test_tracker_rays_parity(dev, h, w, mode, monkeypatch):
    _launch_mode(monkeypatch, mode)
    from oracle import tracker_ref as tr
    from monst3r_slam_amd import tracker as T
    p = syn.tracking_problem(h, w, seed=1)
    cfg = default_config()["tracking"]
    Tf_ref, Trel_ref, it_ref = tr.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"],
                                                         p["T_WCk"], p["Qk"], p["valid"], cfg)
    Tf, Trel, info = T.opt_pose_ray_dist_sim3(_t(p["Xf"], dev), _t(p["Xk"], dev),
                                              _t(p["T_WCf"], dev), _t(p["T_WCk"], dev),
                                              _t(p["Qk"], dev), _t(p["valid"], dev), cfg)
    np.testing.assert_allclose(Trel.cpu().numpy(), Trel_ref, atol=TRACK_TOL, rtol=0)
    np.testing.assert_allclose(Tf.cpu().numpy(), Tf_ref, atol=TRACK_TOL, rtol=0)
    assert abs(int(info[0]) - it_ref) <= 1
    assert int(info[1]) == 0
    if mode == "recovered":
        assert int(info[3]) >= 1, "the forced abort must be recovered by the finish launch"
    else:
        assert int(info[3]) == 0


@pytest.mark.parametrize("mode", list(LAUNCH_MODES))
def test_tracker_calib_parity(dev, mode, monkeypatch):
    _launch_mode(monkeypatch, mode)
    from oracle import tracker_ref as tr
    from monst3r_slam_amd import tracker as T
    p = syn.tracking_problem(96, 128, seed=2)
    cfg = default_config()["tracking"]
    Tf_ref, Trel_ref, it_ref = tr.opt_pose_calib_sim3(
        p["Xf"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"], p["meas_k"], p["valid_meas"],
        p["K"], (p["h"], p["w"]), cfg)
    Tf, Trel, info = T.opt_pose_calib_sim3(
        _t(p["Xf"], dev), _t(p["T_WCf"], dev), _t(p["T_WCk"], dev), _t(p["Qk"], dev),
        _t(p["valid"], dev), _t(p["meas_k"], dev), _t(p["valid_meas"], dev), _t(p["K"], dev),
        (p["h"], p["w"]), cfg)
    np.testing.assert_allclose(Trel.cpu().numpy(), Trel_ref, atol=TRACK_TOL, rtol=0)
    assert abs(int(info[0]) - it_ref) <= 1
    assert (int(info[3]) >= 1) == (mode == "recovered")


def test_tracker_barrier_timeout_recovers(dev, monkeypatch):
    """A barrier poll limit of 0 makes every persistent-launch wait that is not already
    complete time out: whatever the interleaving, the result equals the oracle's and the
    frame is not reported as a Cholesky failure."""
    monkeypatch.setenv("M3S_TRACK_SPIN_LIMIT", "0")
    from oracle import tracker_ref as tr
    from monst3r_slam_amd import tracker as T
    p = syn.tracking_problem(384, 512, seed=4)
    cfg = default_config()["tracking"]
    Tf_ref, Trel_ref, it_ref = tr.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"],
                                                         p["T_WCk"], p["Qk"], p["valid"], cfg)
    Tf, Trel, info = T.opt_pose_ray_dist_sim3(_t(p["Xf"], dev), _t(p["Xk"], dev),
                                              _t(p["T_WCf"], dev), _t(p["T_WCk"], dev),
                                              _t(p["Qk"], dev), _t(p["valid"], dev), cfg)
    np.testing.assert_allclose(Trel.cpu().numpy(), Trel_ref, atol=TRACK_TOL, rtol=0)
    assert int(info[1]) == 0 and abs(int(info[0]) - it_ref) <= 1


def test_tracker_cholesky_failure_reported(dev):
    from monst3r_slam_amd import tracker as T
    p = syn.tracking_problem(32, 32, seed=3)
    cfg = default_config()["tracking"]
    with pytest.raises(T.CholeskyError):
        T.opt_pose_ray_dist_sim3(_t(p["Xf"], dev), _t(p["Xk"], dev), _t(p["T_WCf"], dev),
                                 _t(p["T_WCk"], dev), _t(p["Qk"], dev),
                                 torch.zeros(32 * 32, dtype=torch.bool, device=dev), cfg)
