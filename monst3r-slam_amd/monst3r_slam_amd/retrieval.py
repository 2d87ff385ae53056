"""Keyframe retrieval / loop-closure candidate search on the MI355X.

Drop-in for mast3r_slam/retrieval_database.py:9-166 (`RetrievalDatabase`) and
mast3r_utils.load_retriever (mast3r_utils.py:26-33): `update(frame, add_after_query, k,
min_thresh)` returns the indices of up to k earlier keyframes whose ASMK score exceeds
min_thresh, and (add_after_query) indexes the frame.  Every arithmetic step runs in the HIP
library (csrc/retrieval.hip through include/monst3r_slam_amd.h):

  prep_features   prewhiten -> projector -> l2-norm attention -> top-nfeat -> postwhiten
                  (m3s_retr_affine x3, m3s_retr_rownorm, m3s_topk_select)
  quantize_custom m3s_retr_quantize (fp32 distances + per-row k smallest, fused)
  aggregate       m3s_asmk_aggregate (unique words, residual sums, packed sign bits)
  search          m3s_ivf_search over the device-resident inverted file, m3s_topk_select

The reference keeps the inverted file as per-word numpy arrays on the host and quantises on
the GPU; here it is one flat, image-major device array (entries of a keyframe are appended in
ascending word order, which is also the order the reference's search adds them), so a query
is two launches with no host round trip.  Only the final k indices (and one entry count per
added keyframe) come back to the host, where the reference's return value lives.

The retrieval checkpoint (`..._retrieval_trainingfree.pth`) and its 64k codebook are not
available offline: `synthetic_retrieval_weights` draws seeded weights of the same shapes.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

# mast3r/retrieval/processor.py:92-96
BUILD_PARAMS = {"quantize": {"multiple_assignment": 1}}
QUERY_PARAMS = {"quantize": {"multiple_assignment": 5},
                "similarity": {"similarity_threshold": 0.0, "alpha": 3.0}}


def synthetic_retrieval_weights(enc_dim=1024, hdim=1024, ncent=65536, nfeat=300, seed=0):
    """Seeded stand-in for the retrieval checkpoint + codebook (RetrievalModel with
    prewhiten, hdims=[hdim], postwhiten; featweights='l2norm', model.py:107-136)."""
    g = np.random.default_rng(seed)
    q1, _ = np.linalg.qr(g.standard_normal((enc_dim, enc_dim)))
    q2, _ = np.linalg.qr(g.standard_normal((hdim, hdim)))
    return {
        "pre_m": (0.05 * g.standard_normal(enc_dim)).astype(np.float64),
        "pre_p": (q1 * g.uniform(0.5, 2.0, enc_dim)[None, :]).astype(np.float64),
        "proj_w": (g.standard_normal((hdim, enc_dim)) / np.sqrt(enc_dim)).astype(np.float32),
        "proj_b": (0.01 * g.standard_normal(hdim)).astype(np.float32),
        "post_m": (0.05 * g.standard_normal(hdim)).astype(np.float64),
        "post_p": (q2 * g.uniform(0.5, 2.0, hdim)[None, :]).astype(np.float64),
        "nfeat": nfeat,
        "centroids": g.standard_normal((ncent, hdim)).astype(np.float32),
    }


class RetrievalDatabase:
    """retrieval_database.py:9-166 on device.  weights: dict as synthetic_retrieval_weights."""

    def __init__(self, weights=None, device="cuda", image_capacity=256):
        _lib.load()
        w = weights if weights is not None else synthetic_retrieval_weights()
        self.device = torch.device(device)
        dev = self.device
        f32 = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=dev)  # noqa: E731
        self.pre_m, self.pre_p = f32(w["pre_m"]), f32(w["pre_p"])
        self.proj_wt = f32(np.asarray(w["proj_w"]).T)          # [E][H] for Y = X W
        self.proj_b = f32(w["proj_b"])
        self.post_m, self.post_p = f32(w["post_m"]), f32(w["post_p"])
        self.nfeat = int(w["nfeat"])
        self.centroids = f32(w["centroids"])
        self.ncent, self.dim = self.centroids.shape
        self.enc_dim = self.pre_p.shape[0]
        if self.dim % 32:
            raise ValueError("descriptor dimension must be a multiple of 32")
        self.words32 = self.dim // 32
        self.kf_counter = 0
        self.kf_ids = []
        self.query_dtype = torch.float32
        s = _lib.stream(dev)
        self.cnorm2 = torch.empty(self.ncent, dtype=torch.float32, device=dev)
        _lib.check(_lib.load().m3s_retr_rownorm(_lib.ptr(self.centroids), self.ncent, self.dim, 1,
                                                _lib.ptr(self.cnorm2), s), "m3s_retr_rownorm")
        # word workspaces: flags (zero) and word -> query-row map (-1), restored by the kernels
        self._flags = torch.zeros(self.ncent, dtype=torch.int32, device=dev)
        self._word_map = torch.full((self.ncent,), -1, dtype=torch.int32, device=dev)
        # device inverted file, image-major
        self._img_cap = max(1, int(image_capacity))
        self._ent_cap = self._img_cap * self.nfeat
        self.db_packed = torch.empty((self._ent_cap, self.words32), dtype=torch.int32, device=dev)
        self.db_words = torch.empty(self._ent_cap, dtype=torch.int32, device=dev)
        self.img_start = torch.zeros(self._img_cap + 1, dtype=torch.int32, device=dev)
        self.n_entries = 0

    def reset(self):
        """Empty the database (no keyframes indexed), keeping the weights and workspaces —
        a fresh load_retriever() without re-uploading the codebook."""
        self.kf_counter = 0
        self.kf_ids = []
        self.n_entries = 0
        self.img_start.zero_()

    # ---- retrieval_database.py:25-41 ------------------------------------------------------
    def prep_features(self, backbone_feat):
        """[1,S,E] (bf16 or f32) -> top-nfeat whitened local features [1,nfeat,H] f32."""
        lib, s = _lib.load(), _lib.stream(self.device)
        x = backbone_feat.reshape(-1, backbone_feat.shape[-1])
        _lib.require_cuda(x, names=("backbone_feat",))
        if x.dtype not in (torch.bfloat16, torch.float32):
            x = x.float()
        x = x.contiguous()
        S, E = x.shape
        if E != self.enc_dim:
            raise ValueError(f"backbone feature dim {E} != {self.enc_dim}")
        H = self.dim
        pre = torch.empty((S, E), dtype=torch.float32, device=self.device)
        _lib.check(lib.m3s_retr_affine(_lib.ptr(x), int(x.dtype == torch.bfloat16), E, None,
                                       _lib.ptr(self.pre_m), _lib.ptr(self.pre_p), None, S, E, E,
                                       _lib.ptr(pre), s), "prewhiten")
        proj = torch.empty((S, H), dtype=torch.float32, device=self.device)
        _lib.check(lib.m3s_retr_affine(_lib.ptr(pre), 0, E, None, None, _lib.ptr(self.proj_wt),
                                       _lib.ptr(self.proj_b), S, H, E, _lib.ptr(proj), s),
                   "projector")
        attn = torch.empty(S, dtype=torch.float32, device=self.device)
        _lib.check(lib.m3s_retr_rownorm(_lib.ptr(proj), S, H, 0, _lib.ptr(attn), s), "attention")
        nf = min(self.nfeat, S)
        sel = torch.empty(nf, dtype=torch.int64, device=self.device)
        _lib.check(lib.m3s_topk_select(_lib.ptr(attn), 0, S, nf, 1, _lib.ptr(sel), None, s),
                   "how_select_local")
        out = torch.empty((nf, H), dtype=torch.float32, device=self.device)
        _lib.check(lib.m3s_retr_affine(_lib.ptr(proj), 0, H, _lib.ptr(sel), _lib.ptr(self.post_m),
                                       _lib.ptr(self.post_p), None, nf, H, H, _lib.ptr(out), s),
                   "postwhiten")
        self._last_sel = sel
        return out[None]

    # ---- retrieval_database.py:96-105 -----------------------------------------------------
    def quantize_custom(self, qvecs, params):
        lib, s = _lib.load(), _lib.stream(self.device)
        q = qvecs.contiguous()
        M = q.shape[0]
        k = int(params["quantize"]["multiple_assignment"])
        qn = torch.empty(M, dtype=torch.float32, device=self.device)
        _lib.check(lib.m3s_retr_rownorm(_lib.ptr(q), M, self.dim, 1, _lib.ptr(qn), s), "|q|^2")
        ws = torch.empty(int(lib.m3s_retr_quantize_workspace_bytes(M, self.ncent, k)),
                         dtype=torch.uint8, device=self.device)
        codes = torch.empty((M, k), dtype=torch.int32, device=self.device)
        _lib.check(lib.m3s_retr_quantize(_lib.ptr(q), _lib.ptr(qn), M, _lib.ptr(self.centroids),
                                         _lib.ptr(self.cnorm2), self.ncent, self.dim, k,
                                         _lib.ptr(codes), None, _lib.ptr(ws), s), "quantize")
        return codes

    def aggregate(self, des, codes):
        """ASMKKernel.aggregate_image (binary): packed [n*k][D/32] (first `count` rows valid),
        sorted unique words [n*k], count (device i32[1])."""
        lib, s = _lib.load(), _lib.stream(self.device)
        n, k = codes.shape
        words = torch.empty(n * k, dtype=torch.int32, device=self.device)
        count = torch.empty(1, dtype=torch.int32, device=self.device)
        packed = torch.empty((n * k, self.words32), dtype=torch.int32, device=self.device)
        _lib.check(lib.m3s_asmk_aggregate(_lib.ptr(des), n, self.dim, _lib.ptr(codes), k,
                                          _lib.ptr(self.centroids), self.ncent,
                                          _lib.ptr(self._flags), _lib.ptr(words), _lib.ptr(count),
                                          _lib.ptr(packed), s), "aggregate")
        return packed, words, count

    # ---- retrieval_database.py:75-87 + asmk/inverted_file.py:186-208 ----------------------
    def search_scores(self, packed, words, count):
        """Scores f64 [n_images] of the aggregated query against the inverted file."""
        lib, s = _lib.load(), _lib.stream(self.device)
        n_img = self.kf_counter
        scores = torch.zeros(max(n_img, 1), dtype=torch.float64, device=self.device)
        sim = QUERY_PARAMS["similarity"]
        _lib.check(lib.m3s_ivf_search(_lib.ptr(packed), _lib.ptr(words), _lib.ptr(count),
                                      words.shape[0], _lib.ptr(self.db_packed),
                                      _lib.ptr(self.db_words), _lib.ptr(self.img_start), n_img,
                                      self.dim, float(sim["alpha"]),
                                      float(sim["similarity_threshold"]), _lib.ptr(self._word_map),
                                      _lib.ptr(scores), s), "ivf_search")
        return scores[:n_img]

    def query(self, feat, id=None):
        """Returns (scores f64 [n_images] on device, topk codes [n, 5])."""
        codes = self.quantize_custom(feat, QUERY_PARAMS)
        packed, words, count = self.aggregate(feat, codes)
        return self.search_scores(packed, words, count), codes

    def _grow(self, n_img, n_ent):
        dev = self.device
        if n_img + 1 > self._img_cap:
            cap = max(n_img + 1, int(np.ceil(self._img_cap * 1.5)))
            t = torch.zeros(cap + 1, dtype=torch.int32, device=dev)
            t[: self._img_cap + 1] = self.img_start
            self.img_start, self._img_cap = t, cap
        if n_ent > self._ent_cap:
            cap = max(n_ent, int(np.ceil(self._ent_cap * 1.5)))
            p = torch.empty((cap, self.words32), dtype=torch.int32, device=dev)
            w = torch.empty(cap, dtype=torch.int32, device=dev)
            p[: self.n_entries] = self.db_packed[: self.n_entries]
            w[: self.n_entries] = self.db_words[: self.n_entries]
            self.db_packed, self.db_words, self._ent_cap = p, w, cap

    # ---- retrieval_database.py:89-94, 138-166 ---------------------------------------------
    def add_to_database(self, feat, id=None, topk_codes=None):
        k = int(BUILD_PARAMS["quantize"]["multiple_assignment"])
        if topk_codes is None:
            codes = self.quantize_custom(feat, BUILD_PARAMS)
        else:
            codes = topk_codes[:, :k].contiguous()   # reuse the query's codes (:155-159)
        packed, words, count = self.aggregate(feat, codes)
        m = int(count.item())
        g = self.kf_counter
        self._grow(g + 1, self.n_entries + m)
        self.db_packed[self.n_entries: self.n_entries + m] = packed[:m]
        self.db_words[self.n_entries: self.n_entries + m] = words[:m]
        self.n_entries += m
        self.img_start[g + 1] = self.n_entries
        self.kf_ids.append(g)
        self.kf_counter += 1

    # ---- retrieval_database.py:43-72 ------------------------------------------------------
    def update(self, frame, add_after_query, k, min_thresh=0.0):
        feat_in = frame.feat if hasattr(frame, "feat") else frame
        feat = self.prep_features(feat_in)[0]
        topk_image_inds = []
        topk_codes = None
        if self.kf_counter > 0:
            scores, topk_codes = self.query(feat)
            kk = min(k, self.kf_counter)
            idx = torch.empty(kk, dtype=torch.int64, device=self.device)
            vals = torch.empty(kk, dtype=torch.float64, device=self.device)
            if kk > 0:
                _lib.check(_lib.load().m3s_topk_select(_lib.ptr(scores), 1, scores.shape[0], kk, 1,
                                                       _lib.ptr(idx), _lib.ptr(vals),
                                                       _lib.stream(self.device)), "topk")
            idx_h, vals_h = idx.cpu(), vals.cpu()
            topk_image_inds = idx_h[vals_h > min_thresh].tolist()
            self.last_scores = scores
        if add_after_query:
            self.add_to_database(feat, None, topk_codes)
        return topk_image_inds


def load_retriever(mast3r_model=None, retriever_path=None, device="cuda", weights=None):
    """mast3r_utils.load_retriever (mast3r_utils.py:26-33).  The checkpoint path is accepted
    for signature parity; without network or checkpoints the weights are seeded."""
    if retriever_path is not None and weights is None:
        raise FileNotFoundError(f"retrieval checkpoint loading is not available offline: "
                                f"{retriever_path}; pass weights=")
    return RetrievalDatabase(weights, device=device)
