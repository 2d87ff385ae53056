"""ORACLE — test infrastructure only (imported by tests/, never by the product path).

numpy restatement of the backend factor graph's composition, mast3r_slam/global_opt2.py:
  add_factors          :35-107   Q fusion Qj = sqrt(Qii[b, idx_i2j] * Qji) (and the i side),
                                 valid = valid_match & Q > Q_conf, match fractions, the
                                 "both directions above min_match_frac unless consecutive"
                                 acceptance, the early False on a weak relocalisation edge,
                                 edge bookkeeping by concatenation
  get_unique_kf_idx    :109-110
  prep_two_way_edges   :112-118
  get_poses_points     :120-127  X_canon, T_WC, average confidence C / N (frame.py:126-127)
  solve_GN_rays        :129-166  → oracle.gauss_newton("rays") (gn_ref.c), poses written back
                                 for the unpinned keyframes
It consumes the raw output tuple of monst3r_match_symmetric (idx_i2j, idx_j2i, valid_match_j,
valid_match_i, Qii, Qjj, Qji, Qij) as numpy arrays, so a test can feed it exactly what the
device matcher produced (the matcher itself is pinned bit-exact by test_gpu_matching.py).
"""
import numpy as np

from . import oracle as _o


class FactorGraphRef:
    def __init__(self, cfg):
        self.cfg = cfg
        self.ii = np.zeros(0, np.int64)
        self.jj = np.zeros(0, np.int64)
        self.idx_ii2jj = None
        self.idx_jj2ii = None
        self.valid_match_j = None
        self.valid_match_i = None
        self.Q_ii2jj = None
        self.Q_jj2ii = None

    @staticmethod
    def _cat(a, b):
        return b.copy() if a is None else np.concatenate([a, b])

    def add_factors(self, ii, jj, raw, min_match_frac, is_reloc=False):
        idx_i2j, idx_j2i, vmj, vmi, Qii, Qjj, Qji, Qij = [np.asarray(r) for r in raw]
        b = np.arange(idx_i2j.shape[0])[:, None]
        Qj = np.sqrt(Qii[b, idx_i2j] * Qji).astype(np.float32)
        Qi = np.sqrt(Qjj[b, idx_j2i] * Qij).astype(np.float32)
        valid_j = vmj & (Qj > self.cfg["Q_conf"])
        valid_i = vmi & (Qi > self.cfg["Q_conf"])
        nj = valid_j.shape[1] * valid_j.shape[2]
        ni = valid_i.shape[1] * valid_i.shape[2]
        # torch: int64 count / int → float32 true division
        frac_j = (valid_j.sum(axis=(1, 2)).astype(np.float32) / np.float32(nj))
        frac_i = (valid_i.sum(axis=(1, 2)).astype(np.float32) / np.float32(ni))
        ii, jj = np.asarray(ii, np.int64), np.asarray(jj, np.int64)
        invalid = (np.minimum(frac_j, frac_i) < min_match_frac) & ~(ii == jj - 1)
        if invalid.any() and is_reloc:
            return False
        ok = ~invalid
        self.ii = np.concatenate([self.ii, ii[ok]])
        self.jj = np.concatenate([self.jj, jj[ok]])
        self.idx_ii2jj = self._cat(self.idx_ii2jj, idx_i2j[ok])
        self.idx_jj2ii = self._cat(self.idx_jj2ii, idx_j2i[ok])
        self.valid_match_j = self._cat(self.valid_match_j, vmj[ok])
        self.valid_match_i = self._cat(self.valid_match_i, vmi[ok])
        self.Q_ii2jj = self._cat(self.Q_ii2jj, Qj[ok])
        self.Q_jj2ii = self._cat(self.Q_jj2ii, Qi[ok])
        return bool(ok.sum() > 0)

    def get_unique_kf_idx(self):
        return np.unique(np.concatenate([self.ii, self.jj]))

    def prep_two_way_edges(self):
        return (np.concatenate([self.ii, self.jj]), np.concatenate([self.jj, self.ii]),
                np.concatenate([self.idx_ii2jj, self.idx_jj2ii]),
                np.concatenate([self.valid_match_j, self.valid_match_i]),
                np.concatenate([self.Q_ii2jj, self.Q_jj2ii]))

    def solve_GN_rays(self, X, T_WC, C, N):
        """X [K,n,3], T_WC [K,8], C [K,n,1], N [K] keyframe slabs (numpy); T_WC updated in
        place for the unpinned unique keyframes.  Returns the oracle GN result dict."""
        c = self.cfg
        pin = c["pin"]
        uniq = self.get_unique_kf_idx()
        if uniq.size <= pin:
            return None
        Xs = X[uniq].astype(np.float32)
        Twc = np.ascontiguousarray(T_WC[uniq].astype(np.float32))
        Cs = (C[uniq] / N[uniq].astype(np.float32)[:, None, None]).astype(np.float32)
        ii, jj, idx, vm, Q = self.prep_two_way_edges()
        res = _o.gauss_newton("rays", Twc, Xs, Cs, ii, jj, idx, vm, Q, sig0=c["sigma_ray"],
                              sig1=c["sigma_dist"], C_thresh=c["C_conf"], Q_thresh=c["Q_conf"],
                              max_iter=c["max_iters"], delta_thresh=c["delta_norm"])
        T_WC[uniq[pin:]] = Twc[pin:]
        return res
