"""Headless harness.

SlamLoop: the whole main loop (INIT / TRACKING / RELOC, keyframe append, backend factor
graph + GN, retrieval, relocalisation) in the reference's single-thread order; with the
SceneModel stand-in (scene_slam_run) it regresses ATE over a multi-keyframe sequence.

run_tracking: the TRACKING branch of the reference's main
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


class SlamLoop:
    """The whole main loop, main_monster_slam.py:247-332, with the backend of :81-149 and the
    relocalisation of :20-78 run in the loop's own thread at the points the reference's
    `single_thread` mode waits for them (:310-314, :322-327):

      INIT      monst3r_inference_mono → keyframe 0 appended, backend task queued (:279-290)
      TRACKING  the pair inference vs the last keyframe, FrameTracker2.track's matching /
                pose solve / keyframe fusion (Tracker.track_outputs); a lost frame switches
                to RELOC (:292-299); a new keyframe is the frame itself (its own pointmap,
                the tracked pose, its encoder features) appended to the keyframe store, the
                tracker re-anchored on it (idx_f2k reset, tracker2.py:255-257) and the
                backend run for it (:319-327)
      RELOC     mono inference, then relocalization(): retrieval query, the frame appended
                as a keyframe and add_factors to the retrieved keyframes (strict), on success
                the frame takes the first retrieved keyframe's pose and GN refines the graph;
                on failure the keyframe is popped and the next frame relocalises (:20-78)
      backend   for keyframe idx: the previous keyframe plus the retrieval database's top-k
                (added after the query), add_factors(kf_idx, [idx]*n), solve_GN_rays
                (:101-149)

    The tracker's keyframe fusion (X_canon, C, N) is written back to the keyframe store
    before the backend reads it (tracker2.py:244 writes back every frame; single-threaded
    the two are the same), and the GN-updated pose of the tracked keyframe is read back.
    Pose per frame as main_monster_slam.py records it (all_frames.add_pose): the tracked
    pose, or for a lost / relocalising frame its initial pose (the previous frame's).

    model: a PairModel (or the SceneModel stand-in); mast3r / monst3r: handles whose
    pair_model() returns it (FactorGraph, monst3r_inference_mono); retriever: a
    RetrievalDatabase."""

    def __init__(self, model, mast3r, monst3r, h, w, device, retriever, K=None, buffer=64,
                 cfg=None, group=None):
        from . import global_opt as GO
        from . import parallel as P
        from .config import config as _cfg
        from .frontend import Tracker
        self.cfg = cfg or _cfg
        self.model, self.mast3r, self.monst3r = model, mast3r, monst3r
        self.dev = torch.device(device)
        self.h, self.w = h, w
        self.keyframes = GO.Keyframes(h, w, buffer=buffer, device=device,
                                      feat_dim=model.a.enc_dim)
        # one process per GPU (SPMD, every rank runs this loop): the backend's edge work is
        # sharded (ShardedFactorGraph) and the keyframe pointmaps the tracking rank (0)
        # fused or appended are broadcast before each backend step (all_gather_keyframes)
        self.group = group
        self.world = P._world(group)[0]
        self.graph = (P.ShardedFactorGraph(mast3r, monst3r, self.keyframes, K, device,
                                           group=group) if self.world > 1
                      else GO.FactorGraph(mast3r, monst3r, self.keyframes, K, device))
        self.retriever = retriever
        self.tracker = Tracker(model, self.cfg)
        self.mode = "INIT"
        self.frame_ids, self.poses, self.modes = [], [], []
        self.events = []          # (frame, "new_kf" | "lost" | "reloc_ok" | "reloc_fail", kf)
        self.kf_frame_ids = []
        self._T_last = None

    # ---- helpers ----
    def _frame(self, i, img, T_WC):
        from . import monst3r_utils as U
        shape = torch.tensor([[self.h, self.w]], device=self.dev)
        return U.Frame(i, img, shape, shape, None, T_WC.reshape(1, 8).clone())

    def _append_keyframe(self, fr):
        self.keyframes.append(fr)
        self.kf_frame_ids.append(fr.frame_id)
        return len(self.keyframes) - 1

    def _anchor_tracker(self, idx):
        """The tracker follows keyframe idx (keyframes.last_keyframe())."""
        kf = self.keyframes
        self.tracker.add_keyframe(None, kf.T_WC[idx, 0].clone(), X=kf.X[idx].clone(),
                                  C=kf.C[idx].clone(), feat=kf.feat[idx].clone())
        self.tracker.kf.N.fill_(float(kf._h_N[idx]))
        self._tracked_kf = idx

    def _writeback(self):
        """tracker2.py:244: the fused keyframe back into the store."""
        idx = getattr(self, "_tracked_kf", None)
        if idx is None:
            return
        kf, tk = self.keyframes, self.tracker.kf
        # the tracker's on-device fusion is frame.py's weighted_pointmap mode, the only mode
        # in which N_updates == N (every other mode resets N to 1 while N_updates grows)
        mode = self.tracker.cfg["tracking"]["filtering_mode"]
        if mode != "weighted_pointmap":
            raise NotImplementedError(f"SlamLoop fuses keyframes as weighted_pointmap, not {mode}")
        n_upd = kf._h_Nu[idx] + (int(round(float(tk.N.item()))) - kf._h_N[idx])
        kf.X[idx].copy_(tk.X_canon)
        kf.C[idx].copy_(tk.C)
        kf.set_counts([idx], N=int(round(float(tk.N.item()))), N_updates=n_upd)

    def _refresh_pose(self):
        idx = getattr(self, "_tracked_kf", None)
        if idx is not None:
            self.tracker.kf.T_WC.copy_(self.keyframes.T_WC[idx, 0])

    def _sync(self, idx):
        if self.world > 1:
            from . import parallel as P
            dirty = sorted({idx, getattr(self, "_tracked_kf", idx)})
            P.all_gather_keyframes(self.keyframes, dirty, [0] * len(dirty), self.group)

    def backend(self, idx):
        """run_backend's body for keyframe idx (main_monster_slam.py:101-149)."""
        self._writeback()
        self._sync(idx)
        r = self.cfg["retrieval"]
        kf_idx = [idx - 1 - j for j in range(min(1, idx))]
        kf_idx += self.retriever.update(self.keyframes[idx], add_after_query=True, k=r["k"],
                                        min_thresh=r["min_thresh"])
        kf_idx = sorted(set(kf_idx) - {idx})
        if kf_idx:
            self.graph.add_factors(kf_idx, [idx] * len(kf_idx),
                                   self.cfg["local_opt"]["min_match_frac"])
        self.graph.solve_GN_rays()
        self._refresh_pose()

    def relocalize(self, fr):
        """relocalization() (main_monster_slam.py:20-78) for frame fr (pointmap set)."""
        self._writeback()
        r = self.cfg["retrieval"]
        kf_idx = self.retriever.update(fr, add_after_query=False, k=r["k"],
                                       min_thresh=r["min_thresh"])
        if not kf_idx:
            return False
        n = self._append_keyframe(fr)
        self._sync(n)
        ok = self.graph.add_factors([n] * len(kf_idx), kf_idx,
                                    self.cfg["reloc"]["min_match_frac"],
                                    is_reloc=self.cfg["reloc"]["strict"])
        if not ok:
            # keyframes.pop_last(): the slab row is simply reused by the next append
            self.keyframes.n_size -= 1
            self.kf_frame_ids.pop()
            return False
        self.retriever.update(fr, add_after_query=True, k=r["k"], min_thresh=r["min_thresh"])
        self.keyframes.T_WC[n] = self.keyframes.T_WC[kf_idx[0]].clone()
        self.graph.solve_GN_rays()
        fr.T_WC = self.keyframes.T_WC[n].clone()
        # the tracker follows the new keyframe; its idx_f2k restarts from the identity (the
        # reference keeps the previous keyframe's matches as the next iter_proj seed)
        self._anchor_tracker(n)
        return True

    # ---- one frame (main_monster_slam.py:267-332) ----
    def step(self, i, img):
        from . import monst3r_utils as U
        T0 = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1.0], device=self.dev)
        fr = self._frame(i, img, T0 if self._T_last is None else self._T_last)
        mode = self.mode
        self.modes.append(mode)
        if mode == "INIT":
            X, C = U.monst3r_inference_mono(self.monst3r, fr)
            fr.update_pointmap(X[0], C[0])
            idx = self._append_keyframe(fr)
            self.backend(idx)
            self._anchor_tracker(idx)
            self.mode = "TRACKING"
            self._record(i, fr.T_WC)
            return
        if mode == "TRACKING":
            U._ensure_feat(self.model, fr)
            out = self.model.pair(fr.img, feat_j=self.tracker.kf.feat, feat_i=fr.feat)
            res = self.tracker.track_outputs(out, fr.T_WC.reshape(8))
            self.model.join()
            lost, new_kf = bool(res["lost"].item()), bool(res["new_kf"].item())
            if lost:
                self.mode = "RELOC"
                self.events.append((i, "lost", None))
            else:
                fr.T_WC = res["T_WCf"].reshape(1, 8).clone()
            self._record(i, fr.T_WC)
            if new_kf and not lost:
                n = out["X"].shape[1] * out["X"].shape[2]
                fr.update_pointmap(out["X"][0].reshape(n, 3), out["C"][0].reshape(n, 1))
                self._writeback()
                idx = self._append_keyframe(fr)
                self._anchor_tracker(idx)
                self.backend(idx)
                self.events.append((i, "new_kf", idx))
            return
        # RELOC
        X, C = U.monst3r_inference_mono(self.monst3r, fr)
        fr.update_pointmap(X[0], C[0])
        self._record(i, fr.T_WC)
        if self.relocalize(fr):
            self.mode = "TRACKING"
            self._T_last = fr.T_WC.reshape(8).clone()
            self.events.append((i, "reloc_ok", len(self.keyframes) - 1))
        else:
            self.events.append((i, "reloc_fail", None))

    def _record(self, i, T_WC):
        T = T_WC.reshape(8)
        self._T_last = T.clone()
        self.frame_ids.append(i)
        self.poses.append(T.detach().cpu().numpy())

    def run(self, imgs, timestamps, logdir=None, logfile="traj.txt"):
        for i, img in enumerate(imgs):
            self.step(i, img)
        T_WC = np.stack(self.poses).astype(np.float32)
        if logdir is not None:
            E.save_full_traj(logdir, logfile, np.array(self.frame_ids),
                             [timestamps[i] for i in self.frame_ids], T_WC)
        return T_WC


def scene_slam_run(dev, logdir, n=120, h=96, w=128, period=100, lost_frames=(60,), seed=0):
    """The full loop (SlamLoop) on a SyntheticSequence with the SceneModel stand-in: real
    matching, tracker, keyframe store, FactorGraph, GN and retrieval database.  Returns
    (ATE rmse vs the ground truth, the loop)."""
    from . import retrieval as R
    from .scene_model import SceneHandle, SceneModel
    from .sequence import SyntheticSequence
    seq = SyntheticSequence(n, h, w, device=dev, seed=seed, period=period,
                            lost_frames=lost_frames)
    pm = SceneModel(seq)
    hd = SceneHandle(pm)
    loop = SlamLoop(pm, hd, hd, h, w, dev, R.load_retriever(device=dev))
    ts = [f"{i / 30.0:.6f}" for i in range(n)]
    loop.run([seq.img[i] for i in range(n)], ts, logdir, "est.txt")
    write_ground_truth(logdir, "gt.txt", ts, seq.T_gt_np)
    rmse, _ = E.ate(f"{logdir}/est.txt", f"{logdir}/gt.txt")
    return rmse, loop


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
