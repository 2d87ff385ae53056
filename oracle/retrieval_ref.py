"""ORACLE (test infrastructure only — never imported by the product path): numpy restatement of
the keyframe retrieval path, RetrievalDatabase.update
(mast3r_slam/retrieval_database.py:25-166) and the pieces of its dependencies it runs:

  * Whitener / projector / how_select_local   mast3r/retrieval/model.py:55-104
  * quantize_custom                            retrieval_database.py:96-105
  * ASMKKernel.aggregate_image / similarity    asmk/kernel.py:26-68
  * binarize_and_pack_2D / hamming_cdist_packed asmk/cython/hamming.pyx:77-152
  * asmk_kernel                                asmk/functional.py:96-100
  * IVF.add / IVF.search (use_idf=False)       asmk/inverted_file.py:156-208
  * query params                               mast3r/retrieval/processor.py:92-96

Pinning: packing and hamming distances are checked against the reference's own compiled
hamming module (oracle/Makefile.ref builds asmk/cython/hamming.c into oracle/_ref/) and
against the asmk test's independent numpy definitions (asmk/test/test_hamming.py).  The
asmk package itself cannot be imported here (asmk_method imports faiss, not installed), so
aggregation and the inverted file are restated from their source; the MASt3R retrieval
checkpoint and its codebook are not available offline, so weights and centroids are seeded
random (parity of the arithmetic, not of a trained model).
"""
from __future__ import annotations

import numpy as np

# processor.py:92-96 (asmk_params for build_ivf / query_ivf)
BUILD_MULTIPLE_ASSIGNMENT = 1
QUERY_MULTIPLE_ASSIGNMENT = 5
SIMILARITY_THRESHOLD = 0.0
ALPHA = 3.0


def whiten(x, m, p):
    """Whitener.forward (model.py:62-76): fp64 (x - m) @ p, cast back to the input dtype."""
    y = (x.astype(np.float64) - m.astype(np.float64)) @ p.astype(np.float64)
    return y.astype(x.dtype)


def prep_features(feat, w):
    """RetrievalDatabase.prep_features (retrieval_database.py:25-41) for one frame.
    feat: [S, E] float32; w: dict of pre_m [E], pre_p [E,E], proj_w [H,E], proj_b [H],
    post_m [H], post_p [H,H], nfeat.  Returns top-nfeat whitened features [nfeat, H] and
    the selected token indices (descending attention)."""
    x = whiten(feat.astype(np.float32), w["pre_m"], w["pre_p"])
    proj = (x @ w["proj_w"].T.astype(np.float32) + w["proj_b"]).astype(np.float32)
    attn = np.sqrt((proj.astype(np.float32) ** 2).sum(-1, dtype=np.float32))
    proj_w = whiten(proj, w["post_m"], w["post_p"])
    nfeat = min(int(w["nfeat"]), attn.shape[0])
    order = np.lexsort((np.arange(attn.shape[0]), -attn.astype(np.float64)))[:nfeat]
    return proj_w[order], order, attn


def quantize(q, centroids, k):
    """quantize_custom: (|q|^2 + |c|^2) - 2 q c^T in fp32, the k smallest (ascending,
    ties to the lower index)."""
    q = q.astype(np.float32)
    c = centroids.astype(np.float32)
    d = ((q ** 2).sum(1)[:, None] + (c ** 2).sum(1)[None, :]) - np.float32(2) * (q @ c.T)
    order = np.argsort(d, axis=1, kind="stable")[:, :k]
    return order.astype(np.int64), np.take_along_axis(d, order, 1)


def pack_bits(arr):
    """binarize_and_pack_2D (hamming.pyx:77-110) via the asmk test's own numpy definition
    (test_hamming.py:11-18): bit = x > 0, element 0 of each 32 in the MSB."""
    b = arr > 0
    res = np.empty((b.shape[0], int(np.ceil(b.shape[1] / 32))), dtype=np.uint32)
    packed = np.packbits(b, axis=1).astype(np.uint32)
    packed = np.pad(packed, ((0, 0), (0, 4 - packed.shape[1] % 4)), "constant")
    for i in range(res.shape[1]):
        res[:, i] = ((packed[:, 4 * i] << 24) + (packed[:, 4 * i + 1] << 16)
                     + (packed[:, 4 * i + 2] << 8) + packed[:, 4 * i + 3])
    return res


def hamming_norm(q, vecs):
    """hamming_cdist_packed(q[None], vecs) with normalization = bits (hamming.pyx:34-43):
    int popcount sum / float -> float32."""
    x = np.bitwise_xor(vecs, q[None, :])
    cnt = np.unpackbits(x.view(np.uint8), axis=1).sum(1).astype(np.int64)
    return (cnt.astype(np.float32) / np.float32(q.shape[0] * 32)).astype(np.float32)


def aggregate_image(des, word_ids, centroids):
    """ASMKKernel.aggregate_image with binary=True (kernel.py:26-39)."""
    word_ids = word_ids.reshape(des.shape[0], -1)
    unique_ids = np.unique(word_ids)
    ades = np.empty((unique_ids.shape[0], des.shape[1]), dtype=np.float32)
    for i, word in enumerate(unique_ids):
        ades[i] = (des[(word_ids == word).any(axis=1)] - centroids[word]).sum(0)
    return pack_bits(ades), unique_ids, ades


class IVF:
    """asmk.inverted_file.IVF with use_idf=False (idf = 1, norm_factor = entry counts)."""

    def __init__(self, codebook_size):
        self.vecs = [[] for _ in range(codebook_size)]
        self.imids = [[] for _ in range(codebook_size)]
        self.norm_factor = np.zeros(0)
        self.n_images = 0

    def add(self, des, word_ids, image_id):
        assert image_id >= self.n_images
        self.norm_factor = np.concatenate((self.norm_factor,
                                           np.zeros(image_id + 1 - len(self.norm_factor))))
        self.n_images = max(self.n_images, image_id + 1)
        for d, w in zip(des, word_ids):
            self.vecs[w].append(d)
            self.imids[w].append(image_id)
            self.norm_factor[image_id] += 1

    def search(self, des, word_ids, alpha=ALPHA, thr=SIMILARITY_THRESHOLD):
        """IVF.search + ASMKKernel.similarity + asmk_kernel; returns scores by image id."""
        scores = np.zeros(self.n_images)
        q_norm_factor = np.float32(0)
        for qvec, word in zip(des, word_ids):
            q_norm_factor += np.float32(1.0)
            if not self.imids[word]:
                continue
            vecs = np.stack(self.vecs[word])
            ids = np.asarray(self.imids[word], dtype=np.int64)
            sim = np.float32(-2) * hamming_norm(qvec, vecs) + np.float32(1)
            mask = sim >= thr
            sim = np.power(sim[mask], np.float32(alpha)).astype(np.float32)
            ids = ids[mask]
            sim /= np.sqrt(self.norm_factor[ids])
            scores[ids] += sim
        return scores / np.sqrt(q_norm_factor)


class RetrievalDatabase:
    """RetrievalDatabase.update / query / add_to_database (retrieval_database.py:43-94)."""

    def __init__(self, weights, centroids):
        self.w = weights
        self.centroids = centroids.astype(np.float32)
        self.ivf = IVF(centroids.shape[0])
        self.kf_counter = 0
        self.kf_ids = []

    def update(self, feat, add_after_query, k, min_thresh=0.0):
        des, _, _ = prep_features(feat, self.w)
        topk_image_inds = []
        topk_codes = None
        scores = None
        if self.kf_counter > 0:
            topk_codes, _ = quantize(des, self.centroids, QUERY_MULTIPLE_ASSIGNMENT)
            packed, words, _ = aggregate_image(des, topk_codes, self.centroids)
            scores = self.ivf.search(packed, words)
            kk = min(k, self.ivf.n_images)
            order = np.lexsort((np.arange(scores.shape[0]), -scores))[:kk]
            topk_image_inds = [int(i) for i in order if scores[i] > min_thresh]
        if add_after_query:
            if topk_codes is None:
                codes, _ = quantize(des, self.centroids, BUILD_MULTIPLE_ASSIGNMENT)
            else:
                codes = topk_codes[:, :BUILD_MULTIPLE_ASSIGNMENT]
            packed, words, _ = aggregate_image(des, codes, self.centroids)
            self.ivf.add(packed, words, self.kf_counter)
            self.kf_ids.append(self.kf_counter)
            self.kf_counter += 1
        return topk_image_inds, scores
