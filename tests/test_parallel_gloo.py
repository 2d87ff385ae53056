"""Multi-process keyframe-graph sharding (monst3r_slam_amd/parallel.py) on CPU with the
gloo backend, world_size 2 and 3: the sharded edge records and features must equal the
single-process ones exactly, and the factor-graph acceptance must agree.  The per-edge
inference is replaced by a deterministic CPU stand-in (the HIP path is covered by the
GPU tests); what is tested here is the partitioning, packing and all-gather."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

H, W = 16, 48


def _fake_match(ii, jj, n):
    """Deterministic per-edge record depending only on (i, j)."""
    out = {k: [] for k in ("idx_i2j", "idx_j2i", "valid_match_j", "valid_match_i", "Qj", "Qi")}
    for i, j in zip(ii, jj):
        g = torch.Generator().manual_seed(1000 * int(i) + int(j))
        out["idx_i2j"].append(torch.randint(0, n, (n,), generator=g))
        out["idx_j2i"].append(torch.randint(0, n, (n,), generator=g))
        out["valid_match_j"].append(torch.rand(n, 1, generator=g) < 0.6 + 0.03 * int(i))
        out["valid_match_i"].append(torch.rand(n, 1, generator=g) < 0.5 + 0.02 * int(j))
        out["Qj"].append(torch.rand(n, 1, generator=g) * 4)
        out["Qi"].append(torch.rand(n, 1, generator=g) * 4)
    return {k: torch.stack(v) for k, v in out.items()}


def _graph(cls, **kw):
    from monst3r_slam_amd.global_opt import Keyframes
    frames = Keyframes(H, W, buffer=8, device="cpu")
    for k in range(6):
        frames.img[k] = torch.full((1, 3, H, W), float(k))
        frames.n_size = 6
    g = cls(None, None, frames, device="cpu", **kw)
    g._match_local = lambda ii, jj: _fake_match(ii, jj, H * W)  # noqa: E731
    if not hasattr(cls, "_match_local"):    # single-process graph: stand in directly
        g.match_edges = g._match_local
    return g, frames


EDGES = ([0, 1, 2, 3, 4, 0, 1, 2], [1, 2, 3, 4, 5, 3, 4, 5])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from monst3r_slam_amd import parallel as P
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, frames = _graph(P.ShardedFactorGraph)
        r = g.match_edges(*EDGES)
        added = g.add_factors(*EDGES, min_match_frac=0.3)

        def enc(imgs):  # stand-in encoder: features filled with the keyframe's index
            S = (H // 16) * (W // 16)
            return imgs[:, 0, 0, 0].reshape(-1, 1, 1).expand(-1, S, 1024).to(
                torch.bfloat16), None

        P.shard_keyframe_features(frames, range(6), enc)
        # numpy payloads travel by value: torch tensors would travel as shared-memory handles
        # whose owner may exit before the parent opens them (connection reset)
        loc = {k: getattr(g, k).numpy() for k in ("idx_ii2jj", "idx_jj2ii", "valid_match_j",
                                                  "valid_match_i", "Q_ii2jj", "Q_jj2ii")}
        q.put((rank, {k: v.numpy() for k, v in r.items()}, bool(added), g.ii.numpy(),
               g.jj.numpy(), frames.feat[:6].float().numpy(), g.owner.numpy(), loc,
               g.local_edge_ids().numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_edges_match_single_process(world):
    from monst3r_slam_amd.global_opt import FactorGraph
    ref_g, ref_frames = _graph(FactorGraph)
    ref = ref_g._match_local(*EDGES)
    ref_added = ref_g.add_factors(*EDGES, min_match_frac=0.3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # accepted edges in order, with the rank that matched each (edge e of the call → e % world)
    pairs = list(zip(*EDGES))
    acc = [pairs.index((int(i), int(j))) for i, j in zip(ref_g.ii, ref_g.jj)]
    for rank, r, added, ii, jj, feats, owner, loc, ids in res:
        r = {k: torch.from_numpy(v) for k, v in r.items()}
        ii, jj, feats = torch.from_numpy(ii), torch.from_numpy(jj), torch.from_numpy(feats)
        for k in ref:
            assert torch.equal(r[k], ref[k].to(r[k].dtype)), (rank, k)
        assert added == ref_added
        assert torch.equal(ii, ref_g.ii) and torch.equal(jj, ref_g.jj)
        # records stay on the rank that matched them: this rank's rows are the single-process
        # graph's rows of the accepted edges it owns, in edge order
        assert list(owner) == [e % world for e in acc]
        rows = [k for k, e in enumerate(acc) if e % world == rank]
        for name, v in loc.items():
            assert torch.equal(torch.from_numpy(v), getattr(ref_g, name)[rows]), (rank, name)
        E = len(acc)
        assert list(ids) == rows + [k + E for k in rows]
        # every rank holds every keyframe's features, whoever encoded it
        for k in range(6):
            assert torch.all(feats[k] == float(k)), (rank, k)


def _kf_worker(rank, world, port, q, single):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from monst3r_slam_amd import parallel as P
    from monst3r_slam_amd.global_opt import Keyframes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = Keyframes(H, W, buffer=8, device="cpu")
        frames.n_size = 6
        # every rank starts from its own (stale) copy; rank r is authoritative for the
        # keyframes it owns and writes rank-tagged values into them
        owner = [0] * 6 if single else [0, 1, 0, 0, 1 % world, 2 % world]
        for k in range(6):
            v = 100.0 * rank + k
            frames.X[k] = v
            frames.C[k] = v + 0.5
            frames.N[k] = rank + 1
            # N_updates is its own counter (frame.py update_pointmap: equal to N only in
            # the weighted_pointmap mode) — rank- and keyframe-tagged so a copy of N shows
            frames.N_updates[k] = 10 * (rank + 1) + k
            frames.T_WC[k] = v + 0.25
        P.all_gather_keyframes(frames, range(6), owner)
        q.put((rank, frames.X[:6].numpy(), frames.C[:6].numpy(), frames.N[:6].numpy(),
               frames.T_WC[:6].numpy(), list(frames._h_N[:6]), owner,
               frames.N_updates[:6].numpy(), list(frames._h_Nu[:6])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("single", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_keyframe_pointmaps_all_gathered(world, single):
    """all_gather_keyframes: after the collective every rank holds, for every keyframe,
    the values of the rank that owns it; one owner (the tracking rank) → a broadcast."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kf_worker, args=(r, world, port, q, single))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, X, C, N, T, hN, owner, Nu, hNu in res:
        for k in range(6):
            v = 100.0 * owner[k] + k
            assert (X[k] == v).all() and (C[k] == v + 0.5).all(), (rank, k)
            assert (T[k] == v + 0.25).all() and N[k] == owner[k] + 1 and hN[k] == owner[k] + 1
            nu = 10 * (owner[k] + 1) + k
            assert Nu[k] == nu and hNu[k] == nu, (rank, k, Nu[k], hNu[k])


def test_pack_roundtrip():
    from monst3r_slam_amd import parallel as P
    n = H * W
    r = _fake_match([0, 3], [2, 5], n)
    buf = P.pack_edges(r, n)
    assert buf.shape == (2, P.record_bytes(n)) and P.record_bytes(n) == 18 * n
    u = P.unpack_edges(buf, n)
    for k in r:
        assert torch.equal(u[k], r[k].to(u[k].dtype)), k


def test_acceptance_rule():
    """global_opt2.py:72-85: an edge is dropped when min(match_frac_j, match_frac_i) <
    min_match_frac unless it joins consecutive keyframes."""
    from monst3r_slam_amd.global_opt import FactorGraph
    g, _ = _graph(FactorGraph)
    n = H * W

    def no_matches_one_way(ii, jj):
        rec = _fake_match(ii, jj, n)
        rec["valid_match_j"][:] = False  # zero matches in one direction
        return rec
    g.match_edges = no_matches_one_way
    assert g.add_factors([0, 0], [1, 2], min_match_frac=0.1) is True
    assert g.ii.tolist() == [0] and g.jj.tolist() == [1]   # only the consecutive edge kept
    assert g.add_factors([0], [2], min_match_frac=0.1, is_reloc=True) is False
