"""A perfect-network stand-in for the pair model over a SyntheticSequence (sequence.py), so
the main loop (harness.SlamLoop) runs every real component — matching, the pose solve,
keyframe fusion, the keyframe store, the FactorGraph with its symmetric matching and GN,
the retrieval database — on real geometry, without trained weights (absent offline).

It implements the PairModel interface those components call (`encode`, `pair`, `mono`,
`symmetric`, `join`, `a.patch` / `a.enc_dim`), answering with what a trained network would
regress for the frames involved:
  mono(f)          Xii = Xcam[f] (camera-f pointmap), C_own[f]
  pair(f, k)       Xii = Xcam[f], Xji = T_f^-1 T_k Xcam[k]; D16 (f, k); C / Q own, other of f
  symmetric(i, j)  Xii, Xji = T_i^-1 T_j Xcam[j], Xjj, Xij = T_j^-1 T_i Xcam[i] (4-view order
                   of monst3r_decode_symmetric_batch, monst3r_utils.py:141-184)
Frames are told apart by their encoder features: encode(img) finds the staged image the
pixels belong to and returns a feature set that is a smooth periodic function of the
trajectory phase (tokens = fixed random directions rotated with the phase), so revisits of a
place give near-identical features and the retrieval database finds them; the features of
every frame encoded are registered so pair / symmetric recover the frame index.
"""
from __future__ import annotations

import math

import torch

from .lie import Sim3


class _Arch:
    patch = 16
    enc_dim = 1024


class SceneModel:
    def __init__(self, seq, seed=3):
        self.seq = seq
        self.a = _Arch()
        self.dev = seq.device
        h, w = seq.h, seq.w
        self.S = (h // 16) * (w // 16)
        g = torch.Generator().manual_seed(seed)
        self.base_c = torch.randn(self.S, 1024, generator=g).to(self.dev)
        self.base_s = torch.randn(self.S, 1024, generator=g).to(self.dev)
        # a pixel signature per staged image (its first row's first 16 values, all channels)
        self._sig = seq.img[:, 0, :, 0, :16].reshape(seq.n_frames, -1)
        self._reg = {}
        self.record = None

    # ---- frame identity ----
    def frame_of_img(self, img):
        d = (self._sig - img.reshape(-1, 3, img.shape[-2], img.shape[-1])[:, :, 0, :16]
             .reshape(img.shape[0], -1)[:, None, :].to(self._sig)).abs().sum(-1)
        return d.argmin(-1).tolist()

    def _key(self, feat_row):
        return tuple(feat_row[0, :4].float().tolist())

    def frame_of_feat(self, feat):
        feat = feat.reshape(-1, self.S, 1024)
        return [self._reg[self._key(feat[b])] for b in range(feat.shape[0])]

    # ---- PairModel interface ----
    def encode(self, img, out=None):
        fs = self.frame_of_img(img)
        feats = []
        for f in fs:
            ph = 2.0 * math.pi * f / self.seq.period
            ft = (math.cos(ph) * self.base_c + math.sin(ph) * self.base_s).bfloat16()
            # frames at one place share features: register the first frame seen there
            self._reg.setdefault(self._key(ft), f)
            feats.append(ft)
        feat = torch.stack(feats)
        gh, gw = self.seq.h // 16, self.seq.w // 16
        yy, xx = torch.meshgrid(torch.arange(gh, device=self.dev), torch.arange(gw, device=self.dev),
                                indexing="ij")
        pos = torch.stack([yy, xx], -1).reshape(1, -1, 2).expand(len(fs), -1, -1).contiguous()
        return feat, pos

    def join(self):
        pass

    def _T(self, f):
        return Sim3(self.seq.T_gt[f])

    def _in(self, f, k):
        """Frame k's pointmap expressed in camera f."""
        s = self.seq
        return (self._T(f).inv() * self._T(k)).act(s.Xcam[k])

    def pair(self, img, feat_j=None, feat_i=None, split_heads=False, out=None, img_j=None):
        s = self.seq
        f = self.frame_of_feat(feat_i)[0] if feat_i is not None else self.frame_of_img(img)[0]
        k = self.frame_of_feat(feat_j)[0]
        h, w = s.h, s.w
        X = torch.stack([s.Xcam[f], self._in(f, k)]).reshape(2, h, w, 3)
        # confidences of both views are the pair's (frame f's draws, as m3s_seq_pair_outputs
        # stages them): an unusable frame makes its whole pair unusable
        C = torch.stack([s.C_own[f], s.C_other[f]]).reshape(2, h, w)
        Q = torch.stack([s.Q_own[f], s.Q_other[f]]).reshape(2, h, w)
        D16 = torch.stack([s.D16[f], s.D16[k]]).reshape(2, h, w, 24)
        return dict(X=X.contiguous(), C=C.contiguous(), Q=Q.contiguous(), D16=D16.contiguous(),
                    D=D16.float(), feat_i=feat_i)

    def mono(self, feat, H, W):
        s = self.seq
        f = self.frame_of_feat(feat)[0]
        X = s.Xcam[f].reshape(1, H, W, 3).expand(2, -1, -1, -1).contiguous()
        C = s.C_own[f].reshape(1, H, W).expand(2, -1, -1).contiguous()
        return X, C

    def symmetric(self, feat_i, feat_j, H, W, chunk=4):
        s = self.seq
        fi, fj = self.frame_of_feat(feat_i), self.frame_of_feat(feat_j)
        B = len(fi)
        X = torch.empty((4, B, H, W, 3), device=self.dev)
        C = torch.empty((4, B, H, W), device=self.dev)
        Q = torch.empty((4, B, H, W), device=self.dev)
        D16 = torch.empty((4, B, H, W, 24), dtype=torch.float16, device=self.dev)
        for b, (i, j) in enumerate(zip(fi, fj)):
            # (camera, points of, confidences of): a decode's two views carry the draws of
            # its first frame, as in pair()
            views = ((i, i, s.C_own, s.Q_own, i), (i, j, s.C_other, s.Q_other, i),
                     (j, j, s.C_own, s.Q_own, j), (j, i, s.C_other, s.Q_other, j))
            for v, (cam, src, Cb, Qb, cf) in enumerate(views):
                X[v, b] = (s.Xcam[src] if cam == src else self._in(cam, src)).reshape(H, W, 3)
                C[v, b] = Cb[cf].reshape(H, W)
                Q[v, b] = Qb[cf].reshape(H, W)
                D16[v, b] = s.D16[src].reshape(H, W, 24)
        return dict(X=X, C=C, Q=Q, D16=D16, D=D16.float())


class SceneHandle:
    """The model handle (mast3r / monst3r object) over a SceneModel."""

    def __init__(self, pm):
        self._pm = pm

    def pair_model(self):
        return self._pm
