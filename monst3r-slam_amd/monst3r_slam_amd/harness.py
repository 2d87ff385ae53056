"""Headless tracking harness: the TRACKING branch of the reference's main
loop (main_monster_slam.py:247-332) without the backend/visualisation processes — per frame
`tracker.track` (or `track_outputs` on given pair outputs), the pose recorded for
`save_full_traj` (evaluate.py:110-141), lost frames keeping the previous pose as the
reference's relocalisation wait does not apply, and the TUM trajectory written at the end so
`evaluate.ate` can regress it against ground truth.  Host syncs happen once per frame (the
reference reads `match_info` / `new_kf` on the host every frame as well).
"""
from __future__ import annotations

import numpy as np
import torch

from . import evaluate as E


def run_tracking(tracker, frames, timestamps, logdir, logfile="traj.txt", outputs=False):
    """frames: iterable of images [1,3,H,W] (outputs=False) or of pair-output dicts
    (X, C, D16, Q device tensors; outputs=True).  The keyframe must already be set
    (tracker.add_keyframe).  Returns (T_WC [n, 8] numpy, lost flags [n], new_kf flags [n])."""
    poses, lost, new_kf = [], [], []
    T_prev = None
    for fr in frames:
        res = tracker.track_outputs(fr, T_prev) if outputs else tracker.track(fr, T_prev)
        T = res["T_WCf"].reshape(-1, 8)[0]
        is_lost = bool(res["lost"].item())
        if not is_lost:
            T_prev = T.clone()
        poses.append((T_prev if T_prev is not None else T).detach().cpu().numpy())
        lost.append(is_lost)
        new_kf.append(bool(res["new_kf"].item()))
    T_WC = np.stack(poses).astype(np.float32)
    ids = np.arange(len(poses))
    E.save_full_traj(logdir, logfile, ids, [timestamps[i] for i in ids], T_WC)
    return T_WC, np.array(lost), np.array(new_kf)


def write_ground_truth(logdir, logfile, timestamps, T_gt):
    E.save_full_traj(logdir, logfile, np.arange(len(T_gt)), list(timestamps), np.asarray(T_gt))


def synthetic_run(dev, logdir, n=8, h=96, w=128, seed=0):
    """Track synthetic.tracking_sequence with a perfect-network stand-in for the pair outputs
    and return (ATE rmse, lost flags, estimated T_WC, T_gt)."""
    from . import synthetic as syn
    from .frontend import Tracker
    X_key, frames, T_gt = syn.tracking_sequence(n, h, w, seed)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    tr = Tracker(model=None)
    T0 = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1], dtype=torch.float32, device=dev)
    tr.add_keyframe(None, T0, X=t(X_key), C=torch.full((h * w, 1), 2.0, device=dev),
                    feat=torch.empty(0, device=dev))
    dev_frames = ({k: t(v) for k, v in fr.items()} for fr in frames)
    ts = [f"{i / 30.0:.6f}" for i in range(n)]
    T_WC, lost, _ = run_tracking(tr, dev_frames, ts, logdir, "est.txt", outputs=True)
    write_ground_truth(logdir, "gt.txt", ts, T_gt)
    rmse, _ = E.ate(f"{logdir}/est.txt", f"{logdir}/gt.txt")
    return rmse, lost, T_WC, T_gt
