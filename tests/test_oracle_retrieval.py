"""CPU: the retrieval oracle (oracle/retrieval_ref.py) pinned against the reference's own
compiled hamming module (asmk/cython/hamming.c, built by oracle/Makefile.ref into
oracle/_ref/ when /root/reference is present), the docstring known answers of
asmk/cython/hamming.pyx, and the asmk test's definitions (asmk/test/test_hamming.py); plus
host-logic properties of the inverted file and the database update sequence."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import retrieval_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")


def _ref_hamming():
    if not glob.glob(os.path.join(REF_DIR, "hamming*.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-f", "Makefile.ref"],
                       check=False, capture_output=True)
    if not glob.glob(os.path.join(REF_DIR, "hamming*.so")):
        pytest.skip("reference hamming module not built (reference absent)")
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import hamming
    return hamming


def test_hamming_docstring_known_answers():
    # hamming.pyx:120, :138-140
    q = np.array([3], np.uint32)
    assert R.hamming_norm(q, np.array([[1]], np.uint32))[0] * 32 == 1.0
    a = np.array([[3], [1]], np.uint32)
    b = np.array([[1], [2]], np.uint32)
    d = np.stack([R.hamming_norm(a[i], b) for i in range(2)]) * 32 / 2   # normalization = 2
    np.testing.assert_array_equal(d, [[0.5, 0.5], [0.0, 1.0]])


@pytest.mark.parametrize("dim", [1, 7, 31, 32, 33, 64, 100, 1024])
def test_pack_bits_matches_reference_module(dim):
    hamming = _ref_hamming()
    arr = (np.random.default_rng(dim).random((10, dim)) - 0.5).astype(np.float32)
    arr[0, : min(dim, 3)] = 0.0                       # x > 0 is false at exactly 0
    np.testing.assert_array_equal(R.pack_bits(arr), hamming.binarize_and_pack_2D(arr))


def test_hamming_matches_reference_module():
    hamming = _ref_hamming()
    g = np.random.default_rng(5)
    a = R.pack_bits((g.random((7, 1024)) - 0.5).astype(np.float32))
    b = R.pack_bits((g.random((40, 1024)) - 0.5).astype(np.float32))
    ref = hamming.hamming_cdist_packed(a, b)
    ours = np.stack([R.hamming_norm(a[i], b) for i in range(7)])
    np.testing.assert_array_equal(ours, ref)


def test_aggregate_image_multiple_assignment():
    g = np.random.default_rng(1)
    des = g.standard_normal((20, 64)).astype(np.float32)
    cent = g.standard_normal((16, 64)).astype(np.float32)
    codes, _ = R.quantize(des, cent, 3)
    packed, words, ades = R.aggregate_image(des, codes, cent)
    assert np.array_equal(words, np.unique(codes))
    for i, w in enumerate(words):
        sel = (codes == w).any(1)
        np.testing.assert_allclose(ades[i], (des[sel] - cent[w]).sum(0), rtol=1e-6, atol=1e-6)
    assert packed.shape == (len(words), 2)


def test_quantize_is_nearest_centroids():
    g = np.random.default_rng(2)
    q = g.standard_normal((30, 32)).astype(np.float32)
    c = g.standard_normal((200, 32)).astype(np.float32)
    codes, d = R.quantize(q, c, 5)
    dd = ((q[:, None, :].astype(np.float64) - c[None]) ** 2).sum(-1)
    np.testing.assert_array_equal(codes, np.argsort(dd, 1, kind="stable")[:, :5])
    assert np.all(np.diff(d, axis=1) >= 0)


def _small_weights(seed=0, E=64, H=64, ncent=128, nfeat=20):
    g = np.random.default_rng(seed)
    return {"pre_m": g.standard_normal(E) * 0.05, "pre_p": np.eye(E) * 1.5,
            "proj_w": (g.standard_normal((H, E)) / 8).astype(np.float32),
            "proj_b": np.zeros(H, np.float32), "post_m": np.zeros(H), "post_p": np.eye(H),
            "nfeat": nfeat, "centroids": g.standard_normal((ncent, H)).astype(np.float32)}


def test_database_retrieves_revisited_keyframe():
    """A frame whose features repeat an indexed keyframe's retrieves it first; self-score of
    identical aggregated descriptors = #shared words / sqrt(n_entries * n_query_words)."""
    w = _small_weights()
    db = R.RetrievalDatabase(w, w["centroids"])
    g = np.random.default_rng(3)
    feats = [g.standard_normal((48, 64)).astype(np.float32) for _ in range(5)]
    for f in feats:
        inds, _ = db.update(f, True, 3)
    inds, scores = db.update(feats[2] + 1e-4 * g.standard_normal((48, 64)).astype(np.float32),
                              False, 3)
    assert inds[0] == 2
    assert scores.shape == (5,) and scores[2] == scores.max()
    assert db.kf_counter == 5 and db.kf_ids == [0, 1, 2, 3, 4]


def test_ivf_search_exact_self_score():
    g = np.random.default_rng(4)
    ivf = R.IVF(50)
    packed = R.pack_bits((g.random((6, 64)) - 0.5).astype(np.float32))
    words = np.array([1, 4, 9, 10, 30, 49])
    ivf.add(packed, words, 0)
    s = ivf.search(packed, words)
    np.testing.assert_allclose(s[0], 6 / np.sqrt(6) / np.sqrt(np.float32(6)), rtol=1e-7)
