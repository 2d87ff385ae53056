"""GPU: keyframe-graph inference and backend on the HIP path.

  * PairModel.symmetric (monst3r_decode_symmetric_batch, chunked problem sets) and
    PairModel.mono against goldens from the reference's own modules
    (tests/golden/graph_small.npz), bf16 tolerances as in test_gpu_vit.py;
  * the monst3r_utils drop-in API and FactorGraph end to end (symmetric matching, Q fusion,
    acceptance, GPU GN), consistency-checked against direct kernel calls;
  * the dynamic-mask kernels against the reference's torch formulas."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden", "graph_small.npz")


_LOG = []


@pytest.fixture(autouse=True)
def _bind_log(parity_log):
    _LOG[:] = [parity_log]
    yield


def _check(X, C, D, Q, gX, gC, gD, gQ, tag):
    rel_X = (X - gX).norm(dim=-1) / gX.norm(dim=-1).clamp_min(1e-6)
    rel_C = (C - gC).abs() / gC.abs()
    cos = F.cosine_similarity(D.float(), gD.float(), dim=-1)
    rel_Q = (Q - gQ).abs() / gQ.abs()
    st = dict(X_med=float(rel_X.median()), X_p99=float(rel_X.quantile(0.99)),
              C_med=float(rel_C.median()), D_cos_med=float(cos.median()),
              D_cos_min=float(cos.min()), Q_med=float(rel_Q.median()))
    print(tag, st)
    if _LOG:
        _LOG[0](tag, **st)
    # bf16 MFMA network vs fp32 reference: the tolerances of test_gpu_vit._compare_pair
    assert st["X_med"] < 0.03 and st["X_p99"] < 0.15, st
    assert st["C_med"] < 0.03, st
    assert st["D_cos_med"] > 0.995 and st["D_cos_min"] > 0.9, st
    assert st["Q_med"] < 0.05, st


@pytest.fixture(scope="module")
def small(dev):
    from monst3r_slam_amd import model as Mdl
    g = {k: torch.from_numpy(v).to(dev) for k, v in np.load(G).items()}
    m, _ = Mdl.build(dev, small=True)
    return m, g


@pytest.mark.parametrize("chunk,sym_chunk", [(2, 7), (4, 7), (None, 7), (None, 2)])
def test_symmetric_batch_vs_reference_goldens(small, chunk, sym_chunk):
    """chunk None: PairModel.symmetric's near-equal chunks of at most sym_chunk pairs
    (B = 3: one chunk of 3; sym_chunk 2: chunks of 2 + 1)."""
    m, g = small
    m.sym_chunk = sym_chunk
    H, W = g["imgs"].shape[-2:]
    feats = [m.encode(g["imgs"][k])[0].clone() for k in range(g["imgs"].shape[0])]
    pi = [int(p[0]) for p in g["pairs"]]
    pj = [int(p[1]) for p in g["pairs"]]
    fi = torch.cat([feats[i] for i in pi])
    fj = torch.cat([feats[j] for j in pj])
    out = m.symmetric(fi, fj, H, W, chunk=chunk)    # B = 3: a ragged last chunk at chunk=2
    _check(out["X"], out["C"], out["D"], out["Q"], g["X"], g["C"], g["D"], g["Q"],
           f"symmetric chunk={chunk}")
    assert torch.equal(out["D16"], out["D"].half())


def test_symmetric_slots_equal_pair_inference(small):
    """Slot (ii, ji) of the symmetric batch is the asymmetric pair inference of (i, j);
    slot (jj, ij) that of (j, i) — same kernels, compared at bf16 level."""
    m, g = small
    H, W = g["imgs"].shape[-2:]
    fa = m.encode(g["imgs"][0])[0].clone()
    fb = m.encode(g["imgs"][1])[0].clone()
    sym = m.symmetric(fa, fb, H, W)
    for d, (f1, f2) in enumerate(((fa, fb), (fb, fa))):
        hooks = m.decode(f1[0], f2[0], None, H // 16, W // 16)
        pts, conf, d16, desc, dq = m.heads(hooks, H // 16, W // 16, H, W)
        for s in range(2):
            assert float((sym["X"][2 * d + s, 0] - pts[s]).abs().max()) <= \
                1e-2 * float(pts[s].abs().max())
            assert float((sym["Q"][2 * d + s, 0] - dq[s]).abs().max()) <= \
                1e-2 * float(dq[s].abs().max())


def test_mono_vs_reference_golden(small):
    m, g = small
    H, W = g["imgs"].shape[-2:]
    f = m.encode(g["imgs"][0])[0].clone()
    X, C = m.mono(f, H, W)
    gX, gC = g["mono_X"].reshape(H, W, 3), g["mono_C"].reshape(H, W)
    rel_X = (X[0] - gX).norm(dim=-1) / gX.norm(dim=-1).clamp_min(1e-6)
    rel_C = (C[0] - gC).abs() / gC.abs()
    assert float(rel_X.median()) < 0.03 and float(rel_C.median()) < 0.03


@pytest.fixture(scope="module")
def api(dev):
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import weights as Wt
    mast3r = U.load_mast3r(device=dev, arch=Wt.small(Wt.MAST3R))
    monst3r = U.load_monst3r(device=dev, arch=Wt.small(Wt.MONST3R))
    return U, mast3r, monst3r


def test_api_match_asymmetric_and_symmetric(api, dev):
    from monst3r_slam_amd import matching
    U, mast3r, monst3r = api
    g = {k: torch.from_numpy(v).to(dev) for k, v in np.load(G).items()}
    H, W = g["imgs"].shape[-2:]
    T0 = torch.tensor([[0, 0, 0, 0, 0, 0, 1, 1.0]], device=dev)
    fr = [U.Frame(k, g["imgs"][k], torch.tensor([[H, W]], device=dev),
                  torch.tensor([[H, W]], device=dev), None, T0) for k in range(3)]
    out = U.monst3r_match_asymmetric(mast3r, monst3r, fr[0], fr[1])
    assert len(out) == 8 and out[0].shape == (1, H * W) and out[1].shape == (1, H * W, 1)
    assert out[2].shape == (1, H * W, 3) and out[4].shape == (1, H * W, 1)
    U._ensure_feat(monst3r.pair_model(), fr[2])
    fi = torch.cat([fr[0].feat, fr[1].feat])
    fj = torch.cat([fr[1].feat, fr[2].feat])
    pos = torch.cat([fr[0].pos, fr[1].pos])
    res = U.monst3r_match_symmetric(mast3r, monst3r, fi, pos, fj, pos, [fr[0].img_true_shape] * 2,
                                    [fr[1].img_true_shape] * 2)
    X, C, D, Q = U.monst3r_decode_symmetric_batch(mast3r, monst3r, fi, pos, fj, pos,
                                                  [fr[0].img_true_shape] * 2, None)
    idx, valid = matching.match(torch.cat((X[0], X[2])), torch.cat((X[1], X[3])),
                                torch.cat((D[0], D[2])), torch.cat((D[1], D[3])))
    assert torch.equal(res[0], idx[:2]) and torch.equal(res[1], idx[2:])
    assert torch.equal(res[2], valid[:2]) and torch.equal(res[3], valid[2:])
    assert torch.equal(res[4], Q[0].reshape(2, -1, 1)) and torch.equal(res[7], Q[3].reshape(2, -1, 1))
    Xm, Cm = U.monst3r_inference_mono(monst3r, fr[2])
    assert Xm.shape == (1, H * W, 3) and Cm.shape == (1, H * W, 1)


def test_factor_graph_end_to_end(api, dev):
    """add_factors (symmetric matching + Q fusion + acceptance) then solve_GN_rays on 4
    keyframes: pinned pose unchanged, others finite; records = direct recomputation."""
    from monst3r_slam_amd import global_opt as GO
    from monst3r_slam_amd import parallel as P
    U, mast3r, monst3r = api
    pm = monst3r.pair_model()
    H, W = 48, 64
    gen = torch.Generator(device=dev).manual_seed(11)
    frames = GO.Keyframes(H, W, buffer=8, device=dev, feat_dim=pm.a.enc_dim)
    for k in range(4):
        img = torch.rand(1, 3, H, W, device=dev, generator=gen) * 2 - 1
        T = torch.tensor([[0.01 * k, 0, 0, 0, 0, 0, 1, 1.0]], device=dev)
        f = U.Frame(k, img, torch.tensor([[H, W]], device=dev), torch.tensor([[H, W]], device=dev),
                    None, T)
        X, C = U.monst3r_inference_mono(monst3r, f)
        f.update_pointmap(X[0], C[0])
        frames.append(f)
    graph = P.ShardedFactorGraph(mast3r, monst3r, frames, device=dev)   # world 1 → local
    ii, jj = [0, 1, 2, 0], [1, 2, 3, 2]
    rec = graph.match_edges(ii, jj)
    base = GO.FactorGraph(mast3r, monst3r, frames, device=dev).match_edges(ii, jj)
    for k in rec:
        assert torch.equal(rec[k], base[k]), k
    graph.add_factors(ii, jj, min_match_frac=0.0)
    assert graph.ii.numel() == 4
    T_before = frames.T_WC[:4].clone()
    graph.solve_GN_rays()
    torch.cuda.synchronize()
    assert torch.equal(frames.T_WC[0], T_before[0])        # pin = 1
    assert torch.isfinite(frames.T_WC[:4]).all()


def test_dynamic_mask_kernels(dev):
    from monst3r_slam_amd import monst3r_utils as U
    g = torch.Generator(device=dev).manual_seed(3)
    H, W = 96, 128
    flow = torch.randn(2, H, W, device=dev, generator=g) * 3
    ego = torch.randn(3, H, W, device=dev, generator=g) * 3
    mask = U.dynamic_mask_from_flow(flow, ego, 0.35)
    err = torch.norm(flow - ego[:2], dim=0)                    # monst3r_utils.py:627-636
    norm = (err - err.min()) / (err.max() - err.min())
    ref = norm > 0.35
    ambiguous = (norm - 0.35).abs() < 1e-6
    assert torch.equal(mask[~ambiguous], ref[~ambiguous])
    assert 0 < int(mask.sum()) < H * W
    # apply_dynamic_mask_to_pointmaps (:300-341)
    b = 2
    X = torch.randn(b, H, W, 3, device=dev, generator=g)
    C = torch.rand(b, H, W, device=dev, generator=g) + 1
    D = torch.randn(b, H, W, 24, device=dev, generator=g).half()
    Q = torch.rand(b, H, W, device=dev, generator=g)
    Xo, Co, Do, Qo = U.apply_dynamic_mask_to_pointmaps(X, C, mask, D, Q, 0.0)
    e = mask[None].expand_as(C)
    Cr, Qr, Dr = C.clone(), Q.clone(), D.clone()
    Cr[e] = 0.0
    Qr[e] = 0.0
    Dr[e[..., None].expand_as(Dr)] = 0.0
    assert torch.equal(Co, Cr) and torch.equal(Qo, Qr) and torch.equal(Do, Dr)
    assert torch.equal(Xo, X)


def test_ego_flow_and_get_dynamic_mask(small, dev):
    """Ego-motion flow kernel against a float64 torch statement of the same warp (parity
    with DepthBasedWarping itself is unpinned: its source is absent), then get_dynamic_mask
    end to end with a stand-in RAFT whose flow is the ego flow plus a moving block: the
    block (and only it) is flagged."""
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import synthetic as syn
    m, _ = small
    H, W = 96, 128
    g = torch.Generator(device=dev).manual_seed(11)
    pts = torch.rand(H, W, 3, device=dev, generator=g) + 0.5
    K = torch.from_numpy(syn.intrinsics(H, W)).to(dev)
    Ti = torch.tensor([0.1, -0.05, 0.02, *syn.quat_from_axis_angle([0, 1, 0.2], 0.05), 1.1],
                      dtype=torch.float32, device=dev)
    Tj = torch.tensor([0.0, 0.0, 0.0, 0, 0, 0, 1, 1.0], dtype=torch.float32, device=dev)
    sR, t = U.sim3_relative_matrix(Ti, Tj)
    ego = U.ego_flow(pts, sR, t, K, K)
    yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float64),
                            torch.arange(W, device=dev, dtype=torch.float64), indexing="ij")
    pix = torch.stack([xx, yy, torch.ones_like(xx)], -1)
    d = 1.0 / (1.0 / (pts[..., 2].double() + 1e-6))
    cam = (pix @ torch.linalg.inv(K.double()).t()) * d[..., None]
    proj = (cam @ sR.double().t() + t.double()) @ K.double().t()
    ref = torch.stack([proj[..., 0] / proj[..., 2] - xx, proj[..., 1] / proj[..., 2] - yy])
    assert torch.allclose(ego[:2].double(), ref, atol=2e-3, rtol=1e-4)
    assert bool((ego[2] == 1).all())
    # end to end: frames with K and poses, RAFT stand-in = ego flow of the mono depth + block
    fr_i = U.Frame(0, torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1,
                   torch.tensor([[H, W]]), torch.tensor([[H, W]]), None, T_WC=Ti[None], K=K)
    fr_j = U.Frame(1, torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1,
                   torch.tensor([[H, W]]), torch.tensor([[H, W]]), None, T_WC=Tj[None], K=K)

    class Handle:
        def pair_model(self):
            return m

    Xm, _ = m.mono(m.encode(fr_i.img)[0], H, W)
    ego_i = U.ego_flow(Xm[0], sR, t, K, K)

    def raft(a, b, iters=20, test_mode=True):
        f = ego_i[:2].clone()
        f[:, 20:40, 30:60] += 25.0
        return None, f[None]

    fr_i.feat = None
    mask = U.get_dynamic_mask(Handle(), raft, fr_i, fr_j, threshold=0.35, sam2_predictor=None)
    assert mask.shape == (H, W) and bool(mask[20:40, 30:60].all())
    assert int(mask.sum()) == 20 * 30
    fr_j.K = None
    assert not bool(U.get_dynamic_mask(Handle(), raft, fr_i, fr_j).any())
