"""Trajectory outputs and ATE: host-side I/O around the tracking path.

  as_SE3          mast3r_slam/lietorch_utils.py:6-14 (Sim3 data [t, q xyzw, s] -> [t, q])
  save_traj       mast3r_slam/evaluate.py:24-45 (one TUM line per keyframe,
                  "t x y z qx qy qz qw", timestamps indexed by keyframe.frame_id)
  save_full_traj  mast3r_slam/evaluate.py:110-141 (every tracked frame, sorted by frame id)
  read_tum / ate  TUM-format reader and absolute trajectory error after a Umeyama Sim3 (or
                  SE3) alignment, the metric the reference's evaluation scripts report (evo's
                  `evo_ape tum --align --correct_scale` convention)

Poses are host data here exactly as in the reference (`.cpu().numpy()` before formatting),
so this module is plain numpy; the calibrated branch (Intrinsics.refine_pose_with_calibration)
is out of scope with use_calib.
"""
from __future__ import annotations

import pathlib

import numpy as np


def _host(a):
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.asarray(a)


def as_SE3(T_WC):
    """Sim3 data [..., 8] (t, q xyzw, s) -> SE3 data [N, 7] (t, q): the scale is dropped."""
    d = _host(T_WC).reshape(-1, 8)
    return np.concatenate([d[:, :3], d[:, 3:7]], -1)


def _line(t, se3):
    # numpy scalars of the pose's dtype, formatted by the f-string as the reference's are
    x, y, z, qx, qy, qz, qw = se3.reshape(-1)
    return f"{t} {x} {y} {z} {qx} {qy} {qz} {qw}\n"


def save_traj(logdir, logfile, timestamps, frames, intrinsics=None):
    """evaluate.py:24-45.  frames: a sequence of keyframes with .frame_id and .T_WC (Sim3
    data), e.g. monst3r_utils.Frame / SharedKeyframes items."""
    if intrinsics is not None:
        raise NotImplementedError("use_calib pose refinement is out of scope")
    logdir = pathlib.Path(logdir)
    logdir.mkdir(exist_ok=True, parents=True)
    with open(logdir / logfile, "w") as f:
        for i in range(len(frames)):
            kf = frames[i]
            f.write(_line(timestamps[kf.frame_id], as_SE3(kf.T_WC)))


def save_full_traj(logdir, logfile, frame_ids, timestamps, T_WC, intrinsics=None):
    """evaluate.py:110-141 over the flat all_frames store: frame_ids [N], timestamps [N]
    (strings or numbers, written as given), T_WC [N, 8] Sim3 data; rows sorted by frame id."""
    if intrinsics is not None:
        raise NotImplementedError("use_calib pose refinement is out of scope")
    logdir = pathlib.Path(logdir)
    logdir.mkdir(exist_ok=True, parents=True)
    ids = _host(frame_ids).reshape(-1).astype(np.int64)
    se3 = as_SE3(T_WC)
    order = sorted(range(len(ids)), key=lambda i: ids[i])   # stable, as list.sort
    with open(logdir / logfile, "w") as f:
        for i in order:
            f.write(_line(timestamps[i], se3[i]))


def read_tum(path):
    """-> (timestamps [N] float64, poses [N, 7] float64 t + q xyzw)."""
    rows = [ln.split() for ln in open(path) if ln.strip() and not ln.startswith("#")]
    a = np.array(rows, dtype=np.float64).reshape(-1, 8)
    return a[:, 0], a[:, 1:]


def quat_to_rot(q):
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def umeyama(src, dst, with_scale=True):
    """s, R, t minimising |dst - (s R src + t)|^2 (Umeyama 1991); src, dst [N, 3]."""
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    cov = xd.T @ xs / src.shape[0]
    U, S, Vt = np.linalg.svd(cov)
    E = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        E[2, 2] = -1
    R = U @ E @ Vt
    s = float(np.trace(np.diag(S) @ E) / (xs ** 2).sum(1).mean()) if with_scale else 1.0
    t = mu_d - s * R @ mu_s
    return s, R, t


def associate(t_est, t_ref, max_diff=0.01):
    """Nearest-timestamp association (TUM tools): index pairs with |dt| <= max_diff."""
    pairs = []
    j = 0
    order = np.argsort(t_ref)
    tr = t_ref[order]
    for i, t in enumerate(t_est):
        j = int(np.clip(np.searchsorted(tr, t), 1, len(tr) - 1)) if len(tr) > 1 else 0
        cand = [c for c in (j - 1, j) if 0 <= c < len(tr)]
        best = min(cand, key=lambda c: abs(tr[c] - t))
        if abs(tr[best] - t) <= max_diff:
            pairs.append((i, int(order[best])))
    return pairs


def ate(est_path, ref_path, with_scale=True, max_diff=0.01):
    """Absolute trajectory error (translation RMSE, metres) of a TUM estimate against a TUM
    reference after Sim3 (with_scale) or SE3 alignment.  Returns (rmse, n_associated)."""
    te, pe = read_tum(est_path)
    tr, pr = read_tum(ref_path)
    pairs = associate(te, tr, max_diff)
    if len(pairs) < 3:
        raise ValueError("fewer than 3 associated poses")
    src = np.stack([pe[i, :3] for i, _ in pairs])
    dst = np.stack([pr[j, :3] for _, j in pairs])
    s, R, t = umeyama(src, dst, with_scale)
    err = dst - (s * (R @ src.T).T + t)
    return float(np.sqrt((err ** 2).sum(1).mean())), len(pairs)


def ate_arrays(est_xyz, ref_xyz, with_scale=True):
    """ATE rmse of already associated translations [N, 3] (as `ate`, without the files)."""
    src, dst = np.asarray(est_xyz, np.float64), np.asarray(ref_xyz, np.float64)
    s, R, t = umeyama(src, dst, with_scale)
    err = dst - (s * (R @ src.T).T + t)
    return float(np.sqrt((err ** 2).sum(1).mean()))
