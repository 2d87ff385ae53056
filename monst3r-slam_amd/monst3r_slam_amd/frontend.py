"""Frontend tracking step — mirror of FrameTracker2.track (tracker2.py:70-270) with
use_dynamic_mask=False, on the MI355X path:

  pair inference  monst3r_asymmetric_inference (monst3r_utils.py:255-297) → model.PairModel
  matching        matching.match (matching.py:8-90)                     → matching.match
  glue            Qk, update_pointmap, get_points_poses, valid_opt (tracker2.py:127-213,
                  272-297; frame.py:60-124 'weighted_pointmap')         → torch plumbing
  pose GN         opt_pose_ray_dist_sim3 / opt_pose_calib_sim3          → tracker (fused HIP)
  keyframe update T_CkCf.act(Xkf) + weighted fusion, new-keyframe test (tracker2.py:238-257)

State kept on the device (the reference keeps it in shared-memory tensors, frame.py:243):
keyframe X_canon / C / N / T_WC / cached encoder features.  `track` performs no host
synchronisation except for the returned booleans (read lazily)."""
from __future__ import annotations

import dataclasses
import os

import torch

from . import _lib
from . import matching as M
from . import tracker as T
from .config import config as _config


@dataclasses.dataclass
class KeyframeState:
    X_canon: torch.Tensor   # [N,3] f32
    C: torch.Tensor         # [N,1] f32 (accumulated confidence)
    N: torch.Tensor         # [1] f32 update count (device: graph-capturable)
    T_WC: torch.Tensor      # [8] f32
    feat: torch.Tensor      # [1,S,E] bf16 (MonST3R encoder features)
    img: torch.Tensor       # [1,3,H,W]


def sim3_act(T, X):
    """lietorch Sim3.act on [...,3] points (s R X + t), T = [t, q xyzw, s]."""
    t, q, s = T[:3], T[3:7], T[7]
    uv = 2.0 * torch.cross(q[:3].expand_as(X), X, dim=-1)
    return s * (X + q[3] * uv + torch.cross(q[:3].expand_as(X), uv, dim=-1)) + t


class Tracker:
    def __init__(self, model, cfg=None):
        self.model = model
        self.cfg = cfg or _config
        self.idx_f2k = None
        self.kf = None
        # MASt3R heads on a side stream (local features first): +3 % frames/s in the
        # prefetched pipeline (profiles/r01_ab_lfside_glue.txt); bench.py turns it on
        self.split_heads = False
        # the glue around the pose solve as 3 fused kernels (csrc/glue.hip) instead of the
        # torch restatement below (~25 small launches)
        self.fused_glue = os.environ.get("M3S_FUSED_GLUE", "1") != "0"
        self._glue = None

    def add_keyframe(self, img, T_WC, X=None, C=None, feat=None):
        if feat is None:
            feat, _ = self.model.encode(img)
            feat = feat.clone()
        if X is None:
            out = self.model.pair(img, feat_j=feat)
            n = out["X"].shape[1] * out["X"].shape[2]
            X = out["X"][0].reshape(n, 3).clone()
            C = out["C"][0].reshape(n, 1).clone()
        self.kf = KeyframeState(X, C, torch.ones(1, device=X.device), T_WC.clone(), feat, img)
        self.reset_idx_f2k(X.shape[0], X.device)

    def reset_idx_f2k(self, n, device):
        """tracker2.py:66-67 (None → identity mapping); kept as a persistent buffer so a
        captured graph sees the previous frame's matches."""
        self.idx_f2k = torch.arange(n, device=device, dtype=torch.int64)[None].contiguous()

    def track(self, img, T_WCf_init=None, feat_i=None):
        """One frame.  Returns dict(new_kf, lost, T_WCf, idx_f2k, match_frac, info, ...);
        the scalar flags are device tensors.  feat_i: the frame's encoder features if
        already computed (FramePipeline)."""
        # the MASt3R DPT heads (outputs the tracking never reads) overlap the MonST3R
        # heads, matching and the pose solve on a side stream; joined before returning
        out = self.model.pair(img, feat_j=self.kf.feat, feat_i=feat_i,
                              split_heads=self.split_heads)
        res = self.track_outputs(out, T_WCf_init)
        self.model.join()
        return res

    def track_outputs(self, out, T_WCf_init=None):
        """tracker2.py:127-270 on the pair-inference outputs X [2,H,W,3] (ii, ji), C [2,H,W],
        D16 f16 [2,H,W,24], Q [2,H,W] — everything after monst3r_asymmetric_inference.
        Host-sync free: where the reference returns early (match_frac < min_match_frac,
        :196-198; Cholesky failure, :234-236) the frame is `lost` and the keyframe fusion
        is masked off on the device instead of skipped."""
        cfg_t = self.cfg["tracking"]
        kf = self.kf
        Xii, Xji = out["X"][0:1], out["X"][1:2]
        H, W = Xii.shape[1:3]
        n = H * W
        # matching.match(Xii, Xji, Dii, Dji, idx_init)  (monst3r_utils.py:498-499)
        # tracker2.py:127: the matches become the next frame's seed — written in place
        idx, valid_match = M.match(Xii, Xji, out["D16"][0:1], out["D16"][1:2], self.idx_f2k,
                                   self.cfg["matching"], idx_out=self.idx_f2k)
        idx = idx[0]
        valid_match = valid_match[0]                       # [N,1]
        if self.fused_glue and out["X"].is_contiguous() and out["C"].is_contiguous():
            return self._track_fused(out, idx, valid_match, n, T_WCf_init)
        Qff = out["Q"][0].reshape(n, 1)
        Qkf = out["Q"][1].reshape(n, 1)
        Qk = torch.sqrt(Qff[idx] * Qkf)                    # tracker2.py:130
        # frame.update_pointmap(Xff, Cff) on a fresh frame (N == 0): X_canon = X, C = C
        Xf_canon = out["X"][0].reshape(n, 3)
        Cf = out["C"][0].reshape(n, 1)
        Xkf = out["X"][1].reshape(n, 3)
        Ckf = out["C"][1].reshape(n, 1)
        # get_points_poses (use_calib False): Xf[idx], Xk, Cf[idx], Ck = C/N
        Xf = Xf_canon[idx]
        Ck = kf.C / kf.N
        Cfi = Cf[idx]
        valid_Q = Qk > cfg_t["Q_conf"]
        valid_opt = valid_match & (Cfi > cfg_t["C_conf"]) & (Ck > cfg_t["C_conf"]) & valid_Q
        valid_kf = valid_match & valid_Q
        match_frac = valid_opt.float().mean()
        T_WCf0 = kf.T_WC if T_WCf_init is None else T_WCf_init
        T_WCf, T_CkCf, info = T.opt_pose_ray_dist_sim3(Xf, kf.X_canon, T_WCf0, kf.T_WC, Qk,
                                                       valid_opt, cfg_t, check=False)
        lost = (match_frac < cfg_t["min_match_frac"]) | (info[1] != 0)
        ok = (~lost).float()
        # keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf) — weighted_pointmap (frame.py:105-109)
        Xkk = sim3_act(T_CkCf, Xkf)
        fused = (kf.C * kf.X_canon + Ckf * Xkk) / (kf.C + Ckf)
        kf.X_canon.copy_(torch.where(lost, kf.X_canon, fused))
        kf.C.add_(Ckf * ok)
        kf.N.add_(ok)
        # keyframe selection (tracker2.py:246-257)
        match_frac_k = valid_kf.float().mean()
        sel = torch.zeros(n, dtype=torch.int32, device=idx.device)
        sel.index_add_(0, idx, valid_match[:, 0].int())    # |unique(idx[valid])|, no sort/sync
        unique_frac_f = (sel > 0).sum().float() / n
        new_kf = (torch.minimum(match_frac_k, unique_frac_f) < cfg_t["match_frac_thresh"]) & ~lost
        return dict(new_kf=new_kf, lost=lost, T_WCf=T_WCf, T_CkCf=T_CkCf, idx_f2k=idx,
                    valid_match=valid_match, match_frac=match_frac, info=info,
                    feat_i=out.get("feat_i"), pair=out)


    def _track_fused(self, out, idx, valid_match, n, T_WCf_init):
        """track_outputs' glue on the fused kernels (m3s_track_glue_pre / _post): same
        quantities and the same device-side lost / new-keyframe semantics."""
        cfg_t = self.cfg["tracking"]
        kf = self.kf
        dev = idx.device
        lib = _lib.load()
        g = self._glue
        if g is None or g["n"] != n:
            g = self._glue = dict(
                n=n, Xf=torch.empty((n, 3), dtype=torch.float32, device=dev),
                Qk=torch.empty((n, 1), dtype=torch.float32, device=dev),
                vo=torch.empty((n, 1), dtype=torch.uint8, device=dev),
                ws=torch.empty((lib.m3s_glue_workspace_bytes(n),), dtype=torch.uint8, device=dev),
                flags=torch.zeros(2, dtype=torch.uint8, device=dev),
                fracs=torch.zeros(3, dtype=torch.float32, device=dev))
        vm = valid_match.view(torch.uint8) if valid_match.dtype == torch.bool else valid_match
        s = _lib.stream(dev)
        X, C, Q = out["X"], out["C"], out["Q"].contiguous()
        P = _lib.ptr
        _lib.check(lib.m3s_track_glue_pre(P(X), P(C), P(Q), P(idx), P(vm), P(kf.C), P(kf.N), n,
                                          float(cfg_t["Q_conf"]), float(cfg_t["C_conf"]),
                                          P(g["Xf"]), P(g["Qk"]), P(g["vo"]), P(g["ws"]), s),
                   "track_glue_pre")
        T_WCf0 = kf.T_WC if T_WCf_init is None else T_WCf_init
        T_WCf, T_CkCf, info = T.opt_pose_ray_dist_sim3(g["Xf"], kf.X_canon, T_WCf0, kf.T_WC,
                                                       g["Qk"], g["vo"], cfg_t, check=False)
        _lib.check(lib.m3s_track_glue_post(P(X), P(C), P(idx), P(vm), P(info), P(T_CkCf), n,
                                           float(cfg_t["min_match_frac"]),
                                           float(cfg_t["match_frac_thresh"]), P(kf.X_canon),
                                           P(kf.C), P(kf.N), P(g["flags"]), P(g["fracs"]),
                                           P(g["ws"]), s), "track_glue_post")
        flags = g["flags"].view(torch.bool)
        return dict(new_kf=flags[0], lost=flags[1], T_WCf=T_WCf, T_CkCf=T_CkCf, idx_f2k=idx,
                    valid_match=valid_match, match_frac=g["fracs"][0], info=info,
                    feat_i=out.get("feat_i"), pair=out)


class FramePipeline:
    """Streaming tracking with future frames' encoder prefetched: the MonST3R encoder of a
    future frame depends only on its image, so it runs on a side stream concurrently with
    the current frame's decoders, heads, matching and pose solve (which leave most CUs idle
    at 768 tokens).  Per-frame work and results are those of Tracker.track; only the
    schedule changes.

    group = 1: step(k) tracks the frame encoded by the previous step into buffer k % 2 and
    encodes the next frame into buffer (k + 1) % 2 (24 dependent blocks per step).
    group = g > 1: frames are encoded g at a time (M = g x 768 tokens per GEMM, one
    attention launch for all), the 24 blocks spread over the g steps that track the
    previous group: step k runs part k % g (blocks 24·p/g .. 24·(p+1)/g; part 0 embeds the
    group first, part g-1 ends with enc_norm) of the group that steps
    g·(k // g + 1) .. g·(k // g + 1) + g - 1 track.  Feature slots: group buffer
    (k // g) % 2, row k % g; the graphs repeat with period 2g (`period`).  Frame latency
    +g - 1 steps (features ready before they are needed)."""

    def __init__(self, tracker, shape_hw, side_priority=0, group=1):
        if group not in (1, 2, 3, 4, 6):
            raise ValueError("group must divide the 24 encoder blocks and be <= 6")
        self.tr = tracker
        m = tracker.model
        H, W = shape_hw
        self.shape_hw = (H, W)
        S = (H // m.a.patch) * (W // m.a.patch)
        self.group = group
        self.period = 2 * group
        if group == 1:
            self.feat = [torch.empty((1, S, m.a.enc_dim), dtype=torch.bfloat16, device=m.dev)
                         for _ in range(2)]
        else:
            self.pairs = [torch.empty((group, S, m.a.enc_dim), dtype=torch.bfloat16,
                                      device=m.dev) for _ in range(2)]
            self.feat = [self.pairs[j // group][j % group:j % group + 1]
                         for j in range(2 * group)]
        self.side = torch.cuda.Stream(m.dev, priority=side_priority)

    def slot(self, k):
        """Feature buffer that step k tracks from."""
        return self.feat[k % self.period]

    def next_slot(self, k):
        """Buffer that step k's prefetch completes (group 1: the next frame's)."""
        return self.feat[(k + 1) % 2] if self.group == 1 else None

    def prime(self, img, k=0):
        """Encode the first frame (group g: the first g frames, img [g,3,H,W]) into the
        buffer(s) step k tracks from (on the current stream)."""
        if self.group == 1:
            self.tr.model.encode(img, out=self.feat[k % 2])
        else:
            self.tr.model.encode(img, out=self.pairs[(k // self.group) % 2], concurrent=True)

    def _part(self, img_next, k):
        g = self.group
        H, W = self.shape_hw
        part = k % g
        return self.tr.model.encode_part(
            (g, 3, H, W), part, g, img=img_next if part == 0 else None,
            out=self.pairs[(k // g + 1) % 2] if part == g - 1 else None)

    def encode_side(self, img_next, k):
        """Issue step k's share of the prefetch on the current (side) stream: group 1 the
        whole encoder of img_next [1,3,H,W]; group g its part k % g of the group encode
        (img_next [g,3,H,W] is read by part 0 only)."""
        m = self.tr.model
        if self.group == 1:
            m.encode(img_next, out=self.feat[(k + 1) % 2], concurrent=True)
            return
        self._part(img_next, k)

    def step(self, img_cur, img_next, k, T_WCf_init=None):
        """group 1 only: track img_cur, prefetch img_next."""
        if self.group != 1:
            raise RuntimeError("FramePipeline.step drives group=1; SequenceLoop drives groups")
        main = torch.cuda.current_stream(self.tr.model.dev)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            self.encode_side(img_next, k)
        res = self.tr.track(img_cur, T_WCf_init, feat_i=self.feat[k % 2])
        main.wait_stream(self.side)
        return res
