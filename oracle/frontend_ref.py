"""ORACLE — test infrastructure only.  numpy restatement of the per-frame tracking glue of
FrameTracker2.track (mast3r_slam/tracker2.py:127-270, use_dynamic_mask off, use_calib off)
on given pair-inference outputs, with the C matching oracle (oracle/oracle.py) and the
numpy Sim3 GN (oracle/tracker_ref.py):

  idx_f2k, valid_match = matching.match(Xii, Xji, Dii, Dji, idx_init)      :121-127
  Qk = sqrt(Qff[idx] * Qkf)                                                  :130
  frame.update_pointmap(Xff, Cff) (fresh frame → X_canon = Xff, C = Cff)     :162
  Xf, Cf = X_canon[idx], C[idx]; Ck = C_kf / N_kf  (get_points_poses)        :272-297
  valid_opt = valid_match & Cf > C_conf & Ck > C_conf & Qk > Q_conf          :176-180
  match_frac < min_match_frac → lost (early return, keyframe untouched)      :196-198
  GN (opt_pose_ray_dist_sim3); Cholesky failure → lost                       :200-236
  keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf)  (weighted_pointmap)        :238-244
  new_kf = min(|valid_kf| / n, |unique(idx[valid_match])| / n) < thresh      :246-257
"""
from __future__ import annotations

import numpy as np

from . import oracle as O
from . import tracker_ref as TR


class Keyframe:
    def __init__(self, X, C, T_WC):
        self.X_canon = X.astype(np.float32).copy()
        self.C = C.astype(np.float32).copy()
        self.N = 1.0
        self.T_WC = T_WC.astype(np.float32).copy()


def track_outputs(X, C, D16, Q, kf: Keyframe, idx_init, cfg_m, cfg_t, T_init=None):
    """X [2,H,W,3], C [2,H,W], D16 f16 [2,H,W,24], Q [2,H,W] → dict (mutates kf).
    T_init: the frame's initial pose (the previous frame's, main_monster_slam.py:272-277);
    None → the keyframe's."""
    H, W = X.shape[1:3]
    n = H * W
    idx, valid = O.match(X[0:1], X[1:2], D16[0:1], D16[1:2], idx_init)
    idx, valid = idx[0], valid[0]
    Qff, Qkf = Q[0].reshape(n, 1), Q[1].reshape(n, 1)
    Qk = np.sqrt(Qff[idx] * Qkf).astype(np.float32)
    Xf = X[0].reshape(n, 3)[idx]
    Cf = C[0].reshape(n, 1)[idx]
    Ck = (kf.C / np.float32(kf.N)).astype(np.float32)
    valid_Q = Qk > cfg_t["Q_conf"]
    valid_opt = valid & (Cf > cfg_t["C_conf"]) & (Ck > cfg_t["C_conf"]) & valid_Q
    valid_kf = valid & valid_Q
    match_frac = valid_opt.sum() / valid_opt.size
    res = dict(idx=idx, valid=valid, match_frac=match_frac, lost=False, new_kf=False)
    if match_frac < cfg_t["min_match_frac"]:
        res["lost"] = True
        return res
    try:
        T0 = kf.T_WC if T_init is None else np.asarray(T_init, np.float32)
        T_WCf, T_CkCf, iters = TR.opt_pose_ray_dist_sim3(Xf, kf.X_canon, T0, kf.T_WC,
                                                         Qk[:, 0], valid_opt[:, 0], cfg_t)
    except TR.CholeskyError:
        res["lost"] = True
        return res
    Xkf = X[1].reshape(n, 3)
    Ckf = C[1].reshape(n, 1)
    Xkk = TR.act(T_CkCf, Xkf)
    kf.X_canon = ((kf.C * kf.X_canon + Ckf * Xkk) / (kf.C + Ckf)).astype(np.float32)
    kf.C = (kf.C + Ckf).astype(np.float32)
    kf.N += 1
    match_frac_k = valid_kf.sum() / valid_kf.size
    unique_frac_f = np.unique(idx[valid[:, 0]]).shape[0] / valid_kf.size
    res.update(T_WCf=T_WCf, T_CkCf=T_CkCf, iters=iters,
               new_kf=bool(min(match_frac_k, unique_frac_f) < cfg_t["match_frac_thresh"]))
    return res


class SequenceOracle:
    """The main loop's TRACKING branch bookkeeping (main_monster_slam.py:247-332): the frame
    starts from the previous tracked pose (a lost frame keeps it), a new keyframe is the
    frame itself (keyframes.append(frame): X_canon = Xff, C = Cff, N = 1 after its first
    update_pointmap, T_WC = T_WCf) and resets idx_f2k (tracker2.py:256-257)."""

    def __init__(self, X0, C0, T0, cfg):
        self.kf = Keyframe(X0, C0, T0)
        self.idx = None
        self.T_prev = np.asarray(T0, np.float32).copy()
        self.cfg = cfg

    def step(self, X, C, D16, Q):
        n = X.shape[1] * X.shape[2]
        r = track_outputs(X, C, D16, Q, self.kf, self.idx, self.cfg["matching"],
                          self.cfg["tracking"], T_init=self.T_prev)
        self.idx = r["idx"][None]
        if not r["lost"]:
            self.T_prev = r["T_WCf"].astype(np.float32).copy()
        if r["new_kf"]:
            self.kf = Keyframe(X[0].reshape(n, 3), C[0].reshape(n, 1), r["T_WCf"])
            self.idx = None
        return r
