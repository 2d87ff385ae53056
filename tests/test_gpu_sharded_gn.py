"""GPU: the edge-sharded backend Gauss-Newton (parallel.ShardedFactorGraph.solve_GN_*,
SURVEY §8e; C ABI m3s_gn_sharded_begin / m3s_gn_*_edge_pass / m3s_gn_solve_step) against
the unsharded drop-in (mast3r_slam_backends.gauss_newton_*, itself checked against
oracle/gn_ref.c in test_gpu_c4.py / test_gpu_gn_tracker.py).

World sizes 2 and 3, one process per rank on the box's one GPU, gloo for the per-iteration
all-gather of the E x 35 per-edge sums (staged through the host; RCCL on a real node).
Every rank holds only its own edges' records; the poses must equal the unsharded solve's
BIT FOR BIT (same per-edge sums, same fp64 assembly order), on every rank, for the rays
and the calibrated residual."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
H, W, P, PAIRS = 96, 128, 8, 16


def _scene():
    from monst3r_slam_amd import synthetic as syn
    return syn.keyframe_graph(P=P, h=H, w=W, seed=3, pairs=PAIRS, two_way=True)


def _graph(cls, dev, sc, owner=None, rank=0, **kw):
    from monst3r_slam_amd import global_opt as GO
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    frames = GO.Keyframes(H, W, buffer=P, device=dev, feat_dim=16)
    frames.X[:P] = t(sc["Xs"])
    frames.C[:P] = t(sc["Cs"])
    frames.T_WC[:P] = t(sc["Twc"]).reshape(P, 1, 8)
    frames.set_counts(range(P), N=1)
    frames.set_counts(range(0, P, 3), N=2)
    frames.n_size = P
    g = cls(None, None, frames, K=t(sc["K"].astype(np.float32)), device=dev, **kw)
    E = PAIRS
    rows = list(range(E)) if owner is None else [e for e in range(E) if owner[e] == rank]
    g.ii, g.jj = t(sc["ii"][:E]), t(sc["jj"][:E])
    g.idx_ii2jj, g.idx_jj2ii = t(sc["idx"][:E][rows]), t(sc["idx"][E:][rows])
    g.valid_match_j, g.valid_match_i = t(sc["valid"][:E][rows]), t(sc["valid"][E:][rows])
    g.Q_ii2jj, g.Q_jj2ii = t(sc["Q"][:E][rows]), t(sc["Q"][E:][rows])
    if owner is not None:
        g.owner = torch.as_tensor(owner, dtype=torch.int32, device=dev)
    return g, frames


def _owner(world):
    # uneven ownership: rank 0 holds fewer edges; with world = 3, rank 2 holds none
    if world == 2:
        return [0 if e % 5 == 0 else 1 for e in range(PAIRS)]
    return [0 if e % 3 == 0 else 1 for e in range(PAIRS)]


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from monst3r_slam_amd import parallel as Pm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        g, frames = _graph(Pm.ShardedFactorGraph, dev, _scene(), owner=_owner(world), rank=rank)
        (g.solve_GN_rays if mode == "rays" else g.solve_GN_calib)()
        torch.cuda.synchronize()
        q.put((rank, frames.T_WC[:P].cpu().numpy(), g.gn_iterations))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["rays", "calib"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gn_equals_unsharded(dev, world, mode, parity_log):
    from monst3r_slam_amd.global_opt import FactorGraph
    sc = _scene()
    g, frames = _graph(FactorGraph, dev, sc)
    (g.solve_GN_rays if mode == "rays" else g.solve_GN_calib)()
    ref = frames.T_WC[:P].cpu().numpy()
    assert np.abs(ref - sc["Twc"]).max() > 1e-4          # the solve moved the poses
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, qq, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qq.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, T, iters in res:
        assert np.array_equal(T, ref), (rank, float(np.abs(T - ref).max()))
        assert 1 <= iters <= 10
    parity_log(f"sharded_gn_{mode}_world{world}", pose_maxabs_vs_unsharded=0.0,
               iterations=int(res[0][2]), bar="bit-identical")


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_sharded_solver_one_rank_equals_unsharded(dev, mode):
    """The sharded solver on one rank (the bench's one-GPU keyframe-graph leg calls
    _solve_sharded directly): the rank's slab of per-edge sums is already in two-way edge
    order and goes to the solve as is (no gather / permutation) — poses bit-identical to the
    unsharded solve."""
    from monst3r_slam_amd import parallel as Pm
    from monst3r_slam_amd.global_opt import FactorGraph
    sc = _scene()
    g, frames = _graph(FactorGraph, dev, sc)
    (g.solve_GN_rays if mode == "rays" else g.solve_GN_calib)()
    ref = frames.T_WC[:P].cpu().numpy()
    g1, frames1 = _graph(Pm.ShardedFactorGraph, dev, sc, owner=[0] * PAIRS, rank=0)
    g1._solve_sharded(mode)
    torch.cuda.synchronize()
    assert np.array_equal(frames1.T_WC[:P].cpu().numpy(), ref)
    assert 1 <= g1.gn_iterations <= 10
