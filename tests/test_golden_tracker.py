"""The tracker math pinned to outputs of the REFERENCE's own Python code
(tests/golden/tracker_math.npz, written by tests/golden/make_tracker_goldens.py from
mast3r_slam/geometry.py, nonlinear_optimizer.py and FrameTracker2.opt_pose_*_sim3,
tracker2.py:299-409).

CPU: oracle/tracker_ref.py (the restatement every GPU tracker test checks against) and the
drop-in package's geometry equal the golden vectors.  GPU: the HIP tracker
(monst3r_slam_amd.tracker) reproduces the reference's optimised poses on the golden problems.
"""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tracker_math.npz")
POSE_TOL = 1e-4     # 3-5 f32 GN iterations, reference vs restatement (f32 normal equations)


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


@pytest.fixture(scope="module")
def cfg():
    from monst3r_slam_amd.config import default_config
    return default_config()["tracking"]


def test_ray_dist_and_projection(gold):
    from oracle import tracker_ref as tr
    X = gold["X"]
    ok = np.abs(X).sum(-1) > 1e-3          # rows at the camera centre divide by ~0
    rd, drd = tr.point_to_ray_dist(X, jacobian=True)
    np.testing.assert_allclose(rd[ok], gold["rd"][ok], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(drd[ok], gold["drd"][ok], rtol=1e-5, atol=1e-6)
    pz, J, valid = tr.project_calib(X, gold["K"], (96, 128), -10, 1e-6)
    np.testing.assert_array_equal(valid, gold["pz_valid"])
    front = gold["X"][:, 2] > 1e-2
    np.testing.assert_allclose(pz[front], gold["pz"][front], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(J[front], gold["pz_J"][front], rtol=1e-5, atol=1e-3)
    np.testing.assert_array_equal(pz[~front, 2] == 0, gold["pz"][~front, 2] == 0)


def test_huber_and_convergence(gold, cfg):
    from oracle import tracker_ref as tr
    # torch evaluates the scalar quotient k / |r| to within 1 ulp of numpy's f32 division
    np.testing.assert_allclose(tr.huber(gold["r"], 1.345), gold["huber"], rtol=2.5e-7, atol=0)
    for oc, nc, dn, want in gold["converge_cases"]:
        tau = np.full(7, dn / 7 ** 0.5)
        assert tr.converged(oc, nc, tau, 1e-3, 1e-3) == bool(want), (oc, nc, dn)


def test_constrain_points_to_ray(gold):
    import mast3r_slam.geometry as G
    got = G.constrain_points_to_ray((96, 128), torch.from_numpy(gold["Xs"]),
                                    torch.from_numpy(gold["K"]))
    np.testing.assert_allclose(got.numpy(), gold["Xs_constrained"], rtol=1e-6, atol=1e-6)


def _problem(gold, mode):
    return {k[len(mode) + 1:]: v for k, v in gold.items() if k.startswith(mode + "_")}


def test_oracle_tracker_matches_reference(gold, cfg):
    from oracle import tracker_ref as tr
    p = _problem(gold, "rays")
    Tf, Trel, _ = tr.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"],
                                            p["valid"], cfg)
    np.testing.assert_allclose(Trel, p["T_CkCf_out"], rtol=0, atol=POSE_TOL)
    np.testing.assert_allclose(Tf, p["T_WCf_out"], rtol=0, atol=POSE_TOL)
    p = _problem(gold, "calib")
    Tf, Trel, _ = tr.opt_pose_calib_sim3(p["Xf"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"],
                                         p["meas_k"], p["valid_meas"], p["K"], (96, 128), cfg)
    np.testing.assert_allclose(Trel, p["T_CkCf_out"], rtol=0, atol=POSE_TOL)
    np.testing.assert_allclose(Tf, p["T_WCf_out"], rtol=0, atol=POSE_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_hip_tracker_matches_reference(gold, cfg, mode):
    from monst3r_slam_amd import tracker as T
    dev = torch.device("cuda:0")
    p = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in _problem(gold, mode).items()}
    if mode == "rays":
        Tf, Trel, info = T.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"],
                                                  p["Qk"], p["valid"], cfg)
    else:
        Tf, Trel, info = T.opt_pose_calib_sim3(p["Xf"], p["T_WCf"], p["T_WCk"], p["Qk"],
                                               p["valid"], p["meas_k"], p["valid_meas"], p["K"],
                                               (96, 128), cfg)
    np.testing.assert_allclose(Trel.cpu().numpy(), gold[f"{mode}_T_CkCf_out"], rtol=0,
                               atol=POSE_TOL)
    np.testing.assert_allclose(Tf.cpu().numpy(), gold[f"{mode}_T_WCf_out"], rtol=0,
                               atol=POSE_TOL)
    assert int(info[1]) == 0
