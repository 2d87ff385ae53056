"""CPU: known-answer tests that pin the GN and tracker oracles (synthetic rigid scenes
with known Sim3 motion)."""
import numpy as np

from monst3r_slam_amd import synthetic as syn
from monst3r_slam_amd.config import default_config


def _pose_err(T, T_gt):
    t_err = np.abs(T[:3] - T_gt[:3]).max()
    q = T[3:7] / np.linalg.norm(T[3:7])
    qg = T_gt[3:7] / np.linalg.norm(T_gt[3:7])
    q_err = min(np.abs(q - qg).max(), np.abs(q + qg).max())
    s_err = abs(T[7] - T_gt[7])
    return max(t_err, q_err, s_err)


def test_gn_rays_recovers_trajectory(oracle):
    g = syn.keyframe_graph(P=5, h=24, w=32, seed=0, noise=1e-4)
    Twc = g["Twc"].copy()
    assert max(_pose_err(Twc[k], g["Twc_gt"][k]) for k in range(1, 5)) > 5e-3
    out = oracle.gauss_newton("rays", Twc, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                              g["valid"], g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0,
                              Q_thresh=1.5, max_iter=10, delta_thresh=1e-8)
    assert not out["not_pd"]
    for k in range(5):
        assert _pose_err(Twc[k], g["Twc_gt"][k]) < 2e-3, k


def test_gn_points_recovers_trajectory(oracle):
    g = syn.keyframe_graph(P=4, h=24, w=32, seed=1, noise=1e-4)
    Twc = g["Twc"].copy()
    oracle.gauss_newton("points", Twc, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                        g["valid"], g["Q"], sig0=0.05, C_thresh=0.0, Q_thresh=1.5,
                        max_iter=10, delta_thresh=1e-8)
    for k in range(4):
        assert _pose_err(Twc[k], g["Twc_gt"][k]) < 2e-3, k


def test_gn_singular_system_gives_zero_step(oracle):
    # all matches invalid → H = 0 → Cholesky fails → dx = 0, poses untouched
    g = syn.keyframe_graph(P=3, h=8, w=8, seed=2)
    Twc = g["Twc"].copy()
    before = Twc.copy()
    out = oracle.gauss_newton("rays", Twc, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                              np.zeros_like(g["valid"]), g["Q"], sig0=0.003, sig1=10.0,
                              C_thresh=0.0, Q_thresh=1.5, max_iter=10, delta_thresh=1e-8)
    assert out["not_pd"]
    np.testing.assert_array_equal(out["dx"], 0)
    np.testing.assert_array_equal(Twc, before)
    assert out["iters"] == 1  # ||0|| < thresh → break after the first iteration


def test_tracker_oracle_recovers_relative_pose():
    from oracle import tracker_ref as tr
    p = syn.tracking_problem(96, 128, seed=0, noise=1e-4)
    cfg = default_config()["tracking"]
    T_WCf, T_rel, iters = tr.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"],
                                                    p["Qk"], p["valid"], cfg)
    assert _pose_err(T_rel, p["T_gt"]) < 1e-3
    assert iters < 50
