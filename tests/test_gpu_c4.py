"""GPU: configs[3] at its real size — 16 keyframes, 64 candidate pairs,
384x512 — against the CPU oracle.

  * backend GN rays, P = 16 and E = 128 two-way edges of N = 196608 points, vs gn_ref.c
    (floating point, f32 partial sums in a different order + f64 solve: pose tolerance
    stated below, the measured difference logged to parity_stats.jsonl);
  * FactorGraph.add_factors on the full-size models (symmetric decode of 64 pairs, HIP
    matching) vs oracle/factor_graph_ref.py fed the same raw matcher output: edge lists,
    packed indices, validity and fused Q bit-exact, the acceptance rule and the
    relocalisation early-out;
  * FactorGraph.solve_GN_rays composition (unique keyframes, C / N, two-way packing, pose
    write-back with pin) on the 128 analytic edges vs FactorGraphRef.solve_GN_rays."""
import numpy as np
import pytest
import torch

from monst3r_slam_amd import synthetic as syn
from monst3r_slam_amd.config import default_config

pytestmark = pytest.mark.gpu
H, W, NKF, NPAIRS = 384, 512, 16, 64
POSE_TOL = 5e-5     # 128 edges x 196608 points summed in f32 partials (GPU) vs f64 (oracle)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture(scope="module")
def scene():
    return syn.keyframe_graph(P=NKF, h=H, w=W, seed=21, pairs=NPAIRS, two_way=True)


def test_gn_rays_c4_vs_oracle(oracle, dev, scene, parity_log):
    import mast3r_slam_backends as mb
    g = scene
    assert g["ii"].shape == (2 * NPAIRS,)
    Twc_ref = g["Twc"].copy()
    ref = oracle.gauss_newton("rays", Twc_ref, g["Xs"], g["Cs"], g["ii"], g["jj"], g["idx"],
                              g["valid"], g["Q"], sig0=0.003, sig1=10.0, C_thresh=0.0,
                              Q_thresh=1.5, max_iter=3, delta_thresh=1e-8)
    Twc = _t(g["Twc"], dev)
    (dx,) = mb.gauss_newton_rays(Twc, _t(g["Xs"], dev), _t(g["Cs"], dev), _t(g["ii"], dev),
                                 _t(g["jj"], dev), _t(g["idx"], dev), _t(g["valid"], dev),
                                 _t(g["Q"], dev), 0.003, 10.0, 0.0, 1.5, 3, 1e-8)
    got = Twc.cpu().numpy()
    d = float(np.abs(got - Twc_ref).max())
    parity_log("c4_gn_rays_P16_E128", pose_maxabs=d,
               gt_err_before=float(np.abs(g["Twc"] - g["Twc_gt"]).max()),
               gt_err_after=float(np.abs(got - g["Twc_gt"]).max()))
    assert not ref["not_pd"]
    np.testing.assert_allclose(got, Twc_ref, atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(dx.cpu().numpy(), ref["dx"], atol=POSE_TOL, rtol=0)
    # and the graph actually converged toward the ground truth
    assert np.abs(got - g["Twc_gt"]).max() < 0.1 * np.abs(g["Twc"] - g["Twc_gt"]).max()


def _keyframes(dev, scene, feat_dim):
    from monst3r_slam_amd import global_opt as GO
    gen = torch.Generator(device=dev).manual_seed(5)
    frames = GO.Keyframes(H, W, buffer=NKF, device=dev, feat_dim=feat_dim)
    frames.img[:NKF] = torch.rand(NKF, 1, 3, H, W, device=dev, generator=gen) * 2 - 1
    frames.X[:NKF] = _t(scene["Xs"], dev)
    frames.C[:NKF] = _t(scene["Cs"], dev)
    frames.T_WC[:NKF] = _t(scene["Twc"], dev).reshape(NKF, 1, 8)
    frames.img_true_shape[:NKF] = torch.tensor([[H, W]], dtype=torch.int32, device=dev)
    frames.set_counts(range(NKF), N=1)
    frames.set_counts(range(0, NKF, 3), N=2)          # C / N with N != 1 on some keyframes
    frames.n_size = NKF
    return frames


class _Spy:
    def __init__(self, fn):
        self.fn, self.calls = fn, []

    def __call__(self, *a, **k):
        out = self.fn(*a, **k)
        self.calls.append([o.cpu().numpy() for o in out])
        return out


def test_factor_graph_add_factors_c4_vs_oracle(dev, scene, monkeypatch, parity_log):
    import bench
    from monst3r_slam_amd import global_opt as GO
    from monst3r_slam_amd import model as Mdl
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import parallel as P
    from oracle.factor_graph_ref import FactorGraphRef
    m, _ = Mdl.build(dev)
    h = bench._Bound(m)
    frames = _keyframes(dev, scene, m.a.enc_dim)
    P.shard_keyframe_features(frames, range(NKF), m.encode, None)
    # the pair list the reference's backend builds (bench.retrieval_graph_pairs: previous
    # keyframe + RetrievalDatabase.update top-k hits, main_monster_slam.py:109-130)
    ii, jj, lc, _ = bench.retrieval_graph_pairs([frames.feat[i] for i in range(NKF)], NPAIRS,
                                                device=dev)
    E = len(ii)
    assert E >= 16 and any(lc), (E, sum(lc))     # loop-closure candidates among the pairs
    half = E // 2
    # the networks run (random weights: descriptors and Q are theirs), but their pointmaps
    # are replaced by the scene's geometry — Xii = X_i, Xji = T_i^-1 T_j X_j, Xjj = X_j,
    # Xij = T_j^-1 T_i X_i under the true poses, what a trained network regresses — so the
    # HIP matcher finds real correspondences and the acceptance rule has work to do
    from monst3r_slam_amd.lie import Sim3
    Xs_d = _t(scene["Xs"], dev).reshape(NKF, H, W, 3)
    T_gt = Sim3(_t(scene["Twc_gt"], dev))
    real_decode = U.monst3r_decode_symmetric_batch
    cur = {}

    def geo_decode(*a, **k):
        X, C, D, Q = real_decode(*a, **k)
        X = X.clone()
        for b, (i, j) in enumerate(zip(*cur["e"])):
            X[0, b], X[2, b] = Xs_d[i], Xs_d[j]
            X[1, b] = (T_gt[i].inv() * T_gt[j]).act(Xs_d[j].reshape(-1, 3)).reshape(H, W, 3)
            X[3, b] = (T_gt[j].inv() * T_gt[i]).act(Xs_d[i].reshape(-1, 3)).reshape(H, W, 3)
        return X, C, D, Q

    monkeypatch.setattr(U, "monst3r_decode_symmetric_batch", geo_decode)

    def raw_of(a, b):
        cur["e"] = (a, b)
        shp = [frames.img_true_shape[i] for i in a]
        return [o.cpu().numpy() for o in U.monst3r_match_symmetric(
            h, h, torch.cat([frames.feat[i] for i in a]), torch.cat([frames.pos[i] for i in a]),
            torch.cat([frames.feat[j] for j in b]), torch.cat([frames.pos[j] for j in b]),
            shp, shp)]

    def fused(raw):
        bb = np.arange(raw[0].shape[0])[:, None]
        return (np.sqrt(raw[4][bb, raw[0]] * raw[6]).astype(np.float32),
                np.sqrt(raw[5][bb, raw[1]] * raw[7]).astype(np.float32))

    # random-weight networks: choose Q_conf at the median fused Q of the matched pixels so
    # the per-edge match fractions spread, then a min_match_frac that splits batch 2
    raw1, raw2 = raw_of(ii[:half], jj[:half]), raw_of(ii[half:], jj[half:])
    Qj1, _ = fused(raw1)
    vm_frac = float(raw1[2].mean())
    cfg = default_config()["local_opt"]
    if raw1[2].any():
        cfg["Q_conf"] = float(np.median(Qj1[raw1[2]]))
    monkeypatch.setitem(GO.config, "local_opt", cfg)
    Qj2, Qi2 = fused(raw2)
    fj = (raw2[2] & (Qj2 > cfg["Q_conf"])).mean((1, 2))
    fi = (raw2[3] & (Qi2 > cfg["Q_conf"])).mean((1, 2))
    levels = np.unique(np.minimum(fj, fi).astype(np.float32))
    thr = float(levels[len(levels) // 2])               # accept the upper half of the batch
    spy = _Spy(U.monst3r_match_symmetric)
    monkeypatch.setattr(U, "monst3r_match_symmetric", spy)
    graph = GO.FactorGraph(h, h, frames, device=dev)
    ref = FactorGraphRef(cfg)
    # batch 1: the first half of the pairs, all accepted; batch 2: the rest at the
    # splitting threshold; batch 3: a relocalisation with a weak edge → False, nothing added
    cur["e"] = (ii[:half], jj[:half])
    assert graph.add_factors(ii[:half], jj[:half], 0.0)
    assert ref.add_factors(ii[:half], jj[:half], spy.calls[-1], 0.0)
    for a, c in zip(spy.calls[-1], raw1):                # the matcher is deterministic
        assert np.array_equal(a, c)
    cur["e"] = (ii[half:], jj[half:])
    added = graph.add_factors(ii[half:], jj[half:], thr)
    assert added == ref.add_factors(ii[half:], jj[half:], spy.calls[-1], thr)
    for a, c in zip(spy.calls[-1], raw2):                # the matcher is deterministic
        assert np.array_equal(a, c)
    n_before = graph.ii.numel()
    cur["e"] = ([0, 2], [5, 9])
    assert not graph.add_factors([0, 2], [5, 9], 1.01, is_reloc=True)
    assert not ref.add_factors([0, 2], [5, 9], spy.calls[-1], 1.01, is_reloc=True)
    assert graph.ii.numel() == n_before
    parity_log("c4_add_factors", edges=int(n_before), pairs=E, pairs_from_retrieval=int(sum(lc)),
               threshold=thr, Q_conf=cfg["Q_conf"],
               valid_match_frac=vm_frac,
               match_frac_levels=int(len(levels)),
               matched_frac_median=float(np.median(np.minimum(fj, fi))))
    assert vm_frac > 0.5 and len(levels) > 1
    assert half < n_before < E
    for name in ("ii", "jj", "idx_ii2jj", "idx_jj2ii", "valid_match_j", "valid_match_i",
                 "Q_ii2jj", "Q_jj2ii"):
        got = getattr(graph, name).cpu().numpy()
        want = getattr(ref, name)
        assert got.shape == want.shape and np.array_equal(got, want), name
    assert np.array_equal(graph.get_unique_kf_idx().cpu().numpy(), ref.get_unique_kf_idx())


def test_factor_graph_solve_gn_c4_vs_oracle(dev, scene, monkeypatch, parity_log):
    """The analytic 64-pair graph through FactorGraph (matcher = the scene's exact
    correspondences) and solve_GN_rays vs FactorGraphRef on the same records."""
    from monst3r_slam_amd import global_opt as GO
    from monst3r_slam_amd import monst3r_utils as U
    from oracle.factor_graph_ref import FactorGraphRef
    g = scene
    n = H * W
    E = NPAIRS
    rng = np.random.default_rng(2)
    # raw symmetric outputs for the first 64 (forward) edges of the scene: identity matches,
    # the scene's validity / Q for the two directions, per-view Q
    raw = [g["idx"][:E], g["idx"][E:], g["valid"][:E], g["valid"][E:],
           (1 + 3 * rng.random((E, n, 1))).astype(np.float32),
           (1 + 3 * rng.random((E, n, 1))).astype(np.float32), g["Q"][:E], g["Q"][E:]]

    def fake(*a, **k):
        return tuple(_t(r, dev) for r in raw)

    monkeypatch.setattr(U, "monst3r_match_symmetric", fake)
    frames = _keyframes(dev, scene, 16)
    cfg = default_config()["local_opt"]
    cfg["max_iters"] = 3
    monkeypatch.setitem(GO.config, "local_opt", cfg)
    graph = GO.FactorGraph(None, None, frames, device=dev)
    ref = FactorGraphRef(cfg)
    ii, jj = list(g["ii"][:E]), list(g["jj"][:E])
    assert graph.add_factors(ii, jj, 0.0) and ref.add_factors(ii, jj, raw, 0.0)
    T_ref = g["Twc"].copy()
    N = np.array([2 if k % 3 == 0 else 1 for k in range(NKF)], np.int32)
    res = ref.solve_GN_rays(g["Xs"], T_ref, g["Cs"], N)
    graph.solve_GN_rays()
    got = frames.T_WC[:NKF, 0].cpu().numpy()
    d = float(np.abs(got - T_ref).max())
    parity_log("c4_factor_graph_gn", pose_maxabs=d, oracle_iters=int(res["iters"]))
    assert not res["not_pd"]
    assert np.array_equal(got[0], g["Twc"][0])           # pin = 1
    np.testing.assert_allclose(got, T_ref, atol=POSE_TOL, rtol=0)
