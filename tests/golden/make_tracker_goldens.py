"""Generate the tracker-math golden fixtures FROM THE REFERENCE's own Python code.

Container-only (needs /root/reference; never run on the GPU box).  Executes, from the
reference files, mast3r_slam/geometry.py (point_to_ray_dist, project_calib,
constrain_points_to_ray / backproject, act_Sim3), mast3r_slam/nonlinear_optimizer.py
(huber, check_convergence) and FrameTracker2.opt_pose_ray_dist_sim3 /
opt_pose_calib_sim3 + solve (mast3r_slam/tracker2.py:299-409) on fixed synthetic inputs.
Stand-ins for what the checkout lacks: `lietorch` (git dependency, not installed) →
monst3r_slam_amd.lie (its Sim3 group ops restated from gn_kernels.cu:178-413, itself pinned
to the oracle by tests/test_mast3r_slam_shim.py); `thirdparty.monst3r.third_party.raft`
(absent submodule) → an empty load_RAFT, unused by these functions.  The tracker's control
flow, residuals, Jacobians, Huber weights, normal equations, Cholesky solve and
convergence test are the reference's.

Writes tests/golden/tracker_math.npz.  Run:  python tests/golden/make_tracker_goldens.py
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
REF = "/root/reference/MASt3R-SLAM"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tracker_math.npz")


def _load(rel, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    from monst3r_slam_amd import lie
    from monst3r_slam_amd import synthetic as syn
    from monst3r_slam_amd.config import default_config
    torch.set_grad_enabled(False)
    sys.modules["lietorch"] = lie
    raft = types.ModuleType("thirdparty.monst3r.third_party.raft")
    raft.load_RAFT = lambda *a, **k: None
    for name in ("thirdparty", "thirdparty.monst3r", "thirdparty.monst3r.third_party"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["thirdparty.monst3r.third_party.raft"] = raft
    # tracker2.py's own imports: the reference geometry / nonlinear_optimizer modules (loaded
    # from their files) under their package names; frame / monst3r_utils / config (whose
    # reference versions need skimage, cv2 and the absent MonST3R fork) from the drop-in
    # package — tracker2 uses only their names at import, not in the functions run here
    import mast3r_slam  # noqa: F401  (the drop-in package)
    import mast3r_slam.config as rc
    cfg = default_config()
    rc.config.clear()
    rc.config.update(cfg)
    G = _load("mast3r_slam/geometry.py", "mast3r_slam.geometry")
    NO = _load("mast3r_slam/nonlinear_optimizer.py", "mast3r_slam.nonlinear_optimizer")
    sys.modules["mast3r_slam.geometry"] = G
    sys.modules["mast3r_slam.nonlinear_optimizer"] = NO
    T2 = _load("mast3r_slam/tracker2.py", "ref_tracker2")

    out = {}
    g = torch.Generator().manual_seed(0)
    X = torch.randn(300, 3, generator=g) + torch.tensor([0.0, 0.0, 2.5])
    X[:5, 2] = torch.tensor([-0.5, 1e-7, 0.0, 3.0, 1e-3])      # behind / at the camera
    out["X"] = X.numpy()
    rd, drd = G.point_to_ray_dist(X, jacobian=True)
    out["rd"], out["drd"] = rd.numpy(), drd.numpy()
    K = torch.tensor([[400.0, 0, 64.0], [0, 400.0, 48.0], [0, 0, 1.0]])
    out["K"] = K.numpy()
    pz, J, valid = G.project_calib(X, K, (96, 128), jacobian=True, border=-10, z_eps=1e-6)
    out["pz"], out["pz_J"], out["pz_valid"] = pz.numpy(), J.numpy(), valid.numpy()
    Xs = torch.rand(2, 96 * 128, 3, generator=g) + 0.5
    out["Xs"] = Xs.numpy()
    out["Xs_constrained"] = G.constrain_points_to_ray((96, 128), Xs, K).numpy()
    r = torch.randn(1000, generator=g) * 3
    out["r"], out["huber"] = r.numpy(), NO.huber(r, k=1.345).numpy()
    conv = []
    for oc, nc, dn in ((float("inf"), 5.0, 1e-2), (float("inf"), 5.0, 1e-4), (5.0, 4.999, 1e-2),
                       (5.0, 4.0, 1e-2), (5.0, 4.0, 1e-4)):
        conv.append([oc, nc, dn, float(NO.check_convergence(0, 1e-3, 1e-3, oc, nc,
                                                            torch.full((7,), dn / 7 ** 0.5)))])
    out["converge_cases"] = np.array(conv)

    tr = object.__new__(T2.FrameTracker2)
    tr.cfg = cfg["tracking"]
    for mode, seed in (("rays", 5), ("calib", 6)):
        p = syn.tracking_problem(96, 128, seed=seed)
        t = {k: torch.from_numpy(np.asarray(v)) for k, v in p.items()
             if isinstance(v, np.ndarray)}
        Qk = t["Qk"][:, None].float()
        vld = t["valid"][:, None]
        Twf = lie.Sim3(t["T_WCf"][None].float())
        Twk = lie.Sim3(t["T_WCk"][None].float())
        if mode == "rays":
            Tf, Trel = tr.opt_pose_ray_dist_sim3(t["Xf"].float(), t["Xk"].float(), Twf, Twk, Qk,
                                                 vld)
        else:
            Tf, Trel = tr.opt_pose_calib_sim3(t["Xf"].float(), t["Xk"].float(), Twf, Twk, Qk, vld,
                                              t["meas_k"].float(), t["valid_meas"][:, None],
                                              t["K"].float(), (96, 128))
        for k in ("Xf", "Xk", "Qk", "valid", "T_WCf", "T_WCk", "meas_k", "valid_meas", "K"):
            out[f"{mode}_{k}"] = np.asarray(p[k])
        out[f"{mode}_T_WCf_out"] = Tf.data[0].numpy()
        out[f"{mode}_T_CkCf_out"] = Trel.data[0].numpy()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
