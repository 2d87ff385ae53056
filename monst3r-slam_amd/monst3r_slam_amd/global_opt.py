"""Keyframe store and backend factor graph — mirror of mast3r_slam/frame.py SharedKeyframes
(:243-345) and mast3r_slam/global_opt2.py FactorGraph (:16-221) on the MI355X path.

  Keyframes        device-resident keyframe slabs (X_canon, C, N, T_WC, MonST3R features
                   in bf16, pos, true shape); single process (the reference's
                   torch.multiprocessing shared memory + Manager lock are IPC plumbing, out
                   of scope: SURVEY §2).
  FactorGraph      add_factors → symmetric batched inference + matching of the candidate
                   edges (monst3r_match_symmetric), Q fusion, the edge-acceptance rule, edge
                   bookkeeping; solve_GN_rays / solve_GN_calib → the drop-in
                   mast3r_slam_backends.gauss_newton_* (GPU fp64 solve, in-place poses).
Reference bug kept out: global_opt2.py:54-59 omits the positional `mast3r`
argument of monst3r_match_symmetric; here it is passed, as global_opt.py:49-50 does.

The per-edge inference + matching is `match_edges`, returning one packed record per
candidate edge; `parallel.ShardedFactorGraph` overrides only that method to split the
edges across ranks and all-gather the records.
"""
from __future__ import annotations

import torch

from . import monst3r_utils as U
from .config import config


class Keyframes:
    """SharedKeyframes (frame.py:243-345) without the IPC: fixed-capacity device slabs."""

    def __init__(self, h, w, buffer=64, device="cuda", feat_dim=1024, patch=16):
        self.h, self.w, self.buffer, self.device = h, w, buffer, torch.device(device)
        n, S = h * w, (h // patch) * (w // patch)
        dev = self.device
        self.n_size = 0
        self.dataset_idx = torch.zeros(buffer, dtype=torch.int32, device=dev)
        self.img = torch.zeros(buffer, 1, 3, h, w, device=dev)
        self.img_true_shape = torch.zeros(buffer, 1, 2, dtype=torch.int32, device=dev)
        self.T_WC = torch.zeros(buffer, 1, 8, device=dev)
        self.X = torch.zeros(buffer, n, 3, device=dev)
        self.C = torch.zeros(buffer, n, 1, device=dev)
        self.N = torch.zeros(buffer, dtype=torch.int32, device=dev)
        self.N_updates = torch.zeros(buffer, dtype=torch.int32, device=dev)
        self.feat = torch.zeros(buffer, 1, S, feat_dim, dtype=torch.bfloat16, device=dev)
        self.pos = torch.zeros(buffer, 1, S, 2, dtype=torch.int64, device=dev)
        self.K = torch.zeros(3, 3, device=dev)
        # host mirrors of the per-keyframe counters: __getitem__ needs no device read
        self._h_id = [0] * buffer
        self._h_N = [0] * buffer
        self._h_Nu = [0] * buffer

    def __len__(self):
        return self.n_size

    def set_counts(self, idx, N=1, N_updates=1, frame_id=None):
        """Set the update counts (and dataset index) of keyframes idx (list / range) on the
        device slabs and their host mirrors together (bulk loads that bypass __setitem__)."""
        for i in idx:
            self._h_N[i], self._h_Nu[i] = int(N), int(N_updates)
            if frame_id is not None:
                self._h_id[i] = int(frame_id)
        ix = torch.as_tensor(list(idx), device=self.device)
        self.N[ix] = int(N)
        self.N_updates[ix] = int(N_updates)

    def __getitem__(self, idx) -> U.Frame:
        idx = int(idx)
        f = U.Frame(self._h_id[idx], self.img[idx], self.img_true_shape[idx],
                    self.img_true_shape[idx], None, self.T_WC[idx])
        f.X_canon, f.C, f.feat, f.pos = self.X[idx], self.C[idx], self.feat[idx], self.pos[idx]
        f.N, f.N_updates = self._h_N[idx], self._h_Nu[idx]
        f.K = self.K
        return f

    def __setitem__(self, idx, fr: U.Frame):
        idx = int(idx)
        self._h_id[idx], self._h_N[idx], self._h_Nu[idx] = int(fr.frame_id), int(fr.N), \
            int(fr.N_updates)
        self.dataset_idx[idx] = fr.frame_id
        self.img[idx] = fr.img
        self.img_true_shape[idx] = fr.img_true_shape
        self.T_WC[idx] = _pose_data(fr.T_WC).reshape(1, 8)
        self.X[idx] = fr.X_canon
        self.C[idx] = fr.C
        self.N[idx] = fr.N
        self.N_updates[idx] = fr.N_updates
        if fr.feat is not None:
            self.feat[idx] = fr.feat.reshape(self.feat.shape[1:])
            self.pos[idx] = fr.pos.reshape(self.pos.shape[1:])
        if fr.K is not None:
            self.K[:] = fr.K
        self.n_size = max(self.n_size, idx + 1)

    def append(self, fr: U.Frame):
        self[self.n_size] = fr

    def update_T_WCs(self, T_WCs, idx):
        """frame.py: update_T_WCs — T_WCs [k,1,8] (Sim3 or its data), idx [k]."""
        self.T_WC[idx] = _pose_data(T_WCs).reshape(-1, 1, 8)


def _pose_data(T):
    """Sim3 object (lietorch / monst3r_slam_amd.lie) or raw [..., 8] data → the data."""
    return T.data if not isinstance(T, torch.Tensor) and hasattr(T, "data") else T


class FactorGraph:
    """global_opt2.py:16-221."""

    def __init__(self, mast3r, monst3r, frames: Keyframes, K=None, device="cuda"):
        self.mast3r, self.monst3r, self.frames = mast3r, monst3r, frames
        self.device = torch.device(device)
        self.cfg = config["local_opt"]
        dev = self.device
        self.ii = torch.as_tensor([], dtype=torch.long, device=dev)
        self.jj = torch.as_tensor([], dtype=torch.long, device=dev)
        self.idx_ii2jj = torch.as_tensor([], dtype=torch.long, device=dev)
        self.idx_jj2ii = torch.as_tensor([], dtype=torch.long, device=dev)
        self.valid_match_j = torch.as_tensor([], dtype=torch.bool, device=dev)
        self.valid_match_i = torch.as_tensor([], dtype=torch.bool, device=dev)
        self.Q_ii2jj = torch.as_tensor([], dtype=torch.float32, device=dev)
        self.Q_jj2ii = torch.as_tensor([], dtype=torch.float32, device=dev)
        self.window_size = self.cfg["window_size"]
        self.K = K

    # -- per-edge inference + matching (the part that shards across GPUs) --
    def match_edges(self, ii, jj):
        """Symmetric inference + matching of the edges (ii[e], jj[e]) and the Q fusion of
        global_opt2.py:46-70.  Returns dict of per-edge tensors: idx_i2j, idx_j2i i64 [E,N],
        valid_match_j, valid_match_i bool [E,N,1], Qj, Qi f32 [E,N,1]."""
        kf_ii = [self.frames[i] for i in ii]
        kf_jj = [self.frames[j] for j in jj]
        feat_i = torch.cat([k.feat for k in kf_ii])
        feat_j = torch.cat([k.feat for k in kf_jj])
        pos_i = torch.cat([k.pos for k in kf_ii])
        pos_j = torch.cat([k.pos for k in kf_jj])
        shape_i = [k.img_true_shape for k in kf_ii]
        shape_j = [k.img_true_shape for k in kf_jj]
        (idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij) = \
            U.monst3r_match_symmetric(self.mast3r, self.monst3r, feat_i, pos_i, feat_j, pos_j,
                                      shape_i, shape_j)
        b = torch.arange(idx_i2j.shape[0], device=idx_i2j.device)[:, None].expand_as(idx_i2j)
        Qj = torch.sqrt(Qii[b, idx_i2j] * Qji)
        Qi = torch.sqrt(Qjj[b, idx_j2i] * Qij)
        return dict(idx_i2j=idx_i2j, idx_j2i=idx_j2i, valid_match_j=valid_match_j,
                    valid_match_i=valid_match_i, Qj=Qj, Qi=Qi)

    def add_factors(self, ii, jj, min_match_frac, is_reloc=False):
        """global_opt2.py:35-107: returns True if any edge was added (False early on a
        relocalisation with a weak edge)."""
        r = self.match_edges(ii, jj)
        valid_j = r["valid_match_j"] & (r["Qj"] > self.cfg["Q_conf"])
        valid_i = r["valid_match_i"] & (r["Qi"] > self.cfg["Q_conf"])
        nj = valid_j.shape[1] * valid_j.shape[2]
        ni = valid_i.shape[1] * valid_i.shape[2]
        match_frac_j = valid_j.sum(dim=(1, 2)) / nj
        match_frac_i = valid_i.sum(dim=(1, 2)) / ni
        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        # both directions must clear the threshold; consecutive keyframes always kept
        invalid = torch.minimum(match_frac_j, match_frac_i) < min_match_frac
        invalid = (~(ii_t == (jj_t - 1))) & invalid
        if is_reloc and bool(invalid.any()):
            return False
        ok = ~invalid
        self.ii = torch.cat([self.ii, ii_t[ok]])
        self.jj = torch.cat([self.jj, jj_t[ok]])
        self.idx_ii2jj = torch.cat([self.idx_ii2jj, r["idx_i2j"][ok]])
        self.idx_jj2ii = torch.cat([self.idx_jj2ii, r["idx_j2i"][ok]])
        self.valid_match_j = torch.cat([self.valid_match_j, r["valid_match_j"][ok]])
        self.valid_match_i = torch.cat([self.valid_match_i, r["valid_match_i"][ok]])
        self.Q_ii2jj = torch.cat([self.Q_ii2jj, r["Qj"][ok]])
        self.Q_jj2ii = torch.cat([self.Q_jj2ii, r["Qi"][ok]])
        return bool(ok.sum() > 0)

    def get_unique_kf_idx(self):
        return torch.unique(torch.cat([self.ii, self.jj]), sorted=True)

    def prep_two_way_edges(self):
        ii = torch.cat((self.ii, self.jj), dim=0)
        jj = torch.cat((self.jj, self.ii), dim=0)
        idx_ii2jj = torch.cat((self.idx_ii2jj, self.idx_jj2ii), dim=0)
        valid_match = torch.cat((self.valid_match_j, self.valid_match_i), dim=0)
        Q_ii2jj = torch.cat((self.Q_ii2jj, self.Q_jj2ii), dim=0)
        return ii, jj, idx_ii2jj, valid_match, Q_ii2jj

    def get_poses_points(self, unique_kf_idx):
        """global_opt2.py:120-127 as gathers on the keyframe slabs (no per-keyframe host
        round trip): X_canon, T_WC [P,1,8], average confidence C / N."""
        fr = self.frames
        idx = unique_kf_idx.to(fr.X.device)
        Xs = fr.X[idx]
        T_WCs = fr.T_WC[idx]
        Cs = fr.C[idx] / fr.N[idx].to(fr.C.dtype)[:, None, None]
        return Xs, T_WCs, Cs

    def solve_GN_rays(self):
        """global_opt2.py:129-166."""
        import mast3r_slam_backends
        pin = self.cfg["pin"]
        uniq = self.get_unique_kf_idx()
        if uniq.numel() <= pin:
            return
        Xs, T_WCs, Cs = self.get_poses_points(uniq)
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        pose_data = T_WCs[:, 0, :]
        c = self.cfg
        mast3r_slam_backends.gauss_newton_rays(
            pose_data, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q_ii2jj, c["sigma_ray"],
            c["sigma_dist"], c["C_conf"], c["Q_conf"], c["max_iters"], c["delta_norm"])
        self.frames.update_T_WCs(T_WCs[pin:], uniq[pin:])

    def solve_GN_calib(self):
        """global_opt2.py:168-221 (points constrained to the rays of K first,
        geometry.py:37-42)."""
        import mast3r_slam_backends
        K = self.K
        pin = self.cfg["pin"]
        uniq = self.get_unique_kf_idx()
        if uniq.numel() <= pin:
            return
        Xs, T_WCs, Cs = self.get_poses_points(uniq)
        h, w = self.frames.h, self.frames.w
        Xs = constrain_points_to_ray((h, w), Xs, K)
        ii, jj, idx_ii2jj, valid_match, Q_ii2jj = self.prep_two_way_edges()
        pose_data = T_WCs[:, 0, :]
        c = self.cfg
        mast3r_slam_backends.gauss_newton_calib(
            pose_data, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q_ii2jj, h, w,
            c["pixel_border"], c["depth_eps"], c["sigma_pixel"], c["sigma_depth"], c["C_conf"],
            c["Q_conf"], c["max_iters"], c["delta_norm"])
        self.frames.update_T_WCs(T_WCs[pin:], uniq[pin:])


def constrain_points_to_ray(img_size, Xs, K):
    """geometry.py:37-42 with get_pixel_coords (:116-123) and backproject (:107-114):
    X ← z · ((u - cx)/fx, (v - cy)/fy, 1) per pixel, z = X[..., 2]."""
    h, w = img_size
    v, u = torch.meshgrid(torch.arange(h, device=Xs.device, dtype=Xs.dtype),
                          torch.arange(w, device=Xs.device, dtype=Xs.dtype), indexing="ij")
    tmp1 = ((u - K[0, 2]) / K[0, 0]).reshape(-1)
    tmp2 = ((v - K[1, 2]) / K[1, 1]).reshape(-1)
    z = Xs[..., 2]
    return torch.stack((z * tmp1, z * tmp2, z * 1.0), dim=-1)
