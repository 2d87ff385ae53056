"""Keyframe-graph work sharded over the GPUs of one node.

Tracking is sequential (frame t needs the pose and matches of t-1), so it runs as
independent replicas.  The keyframe graph is data-parallel: every candidate edge's
symmetric inference (4 directed decodes + 8 heads) and its two matchings are
independent, and so is every keyframe's encoder pass.  One process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI on the MI355X node, "gloo" in the
CPU tests):

  shard_keyframe_features  keyframes encoded round-robin across ranks, features
                           all-gathered (1.5 MB bf16 per keyframe at 384x512)
  ShardedFactorGraph       FactorGraph whose add_factors matches the rank's round-robin
                           share of the edges and KEEPS their records (idx, valid, Q:
                           18 B/pixel) on that rank: only the per-edge match fractions are
                           all-gathered for the acceptance rule.  Its GN shards the edge
                           pass the same way — each rank reduces its own edges to 35 f64
                           sums per two-way edge, one E x 35 all-gather per iteration, then
                           the same fp64 solve + retraction on every rank (bit-identical to
                           the unsharded poses).  match_edges (the base-class contract:
                           every record everywhere) all-gathers packed records instead.
  all_gather_keyframes     the keyframe pointmaps (X_canon, C, N, T_WC) each rank is
                           authoritative for — the tracking rank's fused keyframes, new
                           keyframes — all-gathered into every rank's keyframe store before
                           the backend reads them (3.1 MB per keyframe at 384x512), so the
                           replicated GN sees the same pointmaps everywhere
Each all-gather moves ceil(E/world) rows per rank in ONE collective (padded): no per-edge
messages.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from .global_opt import FactorGraph

_FIELDS = (("idx_i2j", torch.int32, 1), ("idx_j2i", torch.int32, 1),
           ("valid_match_j", torch.uint8, 1), ("valid_match_i", torch.uint8, 1),
           ("Qj", torch.float32, 1), ("Qi", torch.float32, 1))


def _world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def record_bytes(n):
    """Bytes of one packed edge record for n pixels."""
    return sum(torch.empty((), dtype=dt).element_size() * c for _, dt, c in _FIELDS) * n


def pack_edges(r, n):
    """dict of per-edge tensors ([E,N] / [E,N,1]) → uint8 [E, record_bytes(n)]."""
    E = r["idx_i2j"].shape[0]
    parts = []
    for name, dt, _ in _FIELDS:
        t = r[name].reshape(E, n).to(dt).contiguous()
        parts.append(t.view(torch.uint8).reshape(E, -1))
    return torch.cat(parts, 1)


def unpack_edges(buf, n):
    """Inverse of pack_edges, back to the FactorGraph.match_edges dtypes/shapes."""
    E = buf.shape[0]
    out, off = {}, 0
    for name, dt, _ in _FIELDS:
        nb = torch.empty((), dtype=dt).element_size() * n
        t = buf[:, off:off + nb].contiguous().view(dt).reshape(E, n)
        off += nb
        if name.startswith("idx"):
            out[name] = t.to(torch.int64)
        elif name.startswith("valid"):
            out[name] = t.bool().unsqueeze(-1)
        else:
            out[name] = t.unsqueeze(-1)
    return out


def all_gather_rows(local, rows_total, group=None):
    """Rows distributed round-robin (row e on rank e % world at slot e // world), each rank
    holding ceil(rows_total / world) slots → [rows_total, ...] in row order on every rank.
    One all-gather of equal-size padded buffers."""
    world, _ = _world(group)
    if world == 1:
        return local[:rows_total]
    gathered = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(gathered, local.contiguous(), group=group)
    per = local.shape[0]
    stacked = torch.stack(gathered, 1).reshape(world * per, *local.shape[1:])  # slot-major
    return stacked[:rows_total]


def shard_keyframe_features(frames, idx, encode, group=None):
    """Encode keyframes idx round-robin across ranks and all-gather the features into
    frames.feat / frames.pos on every rank.  encode(imgs [k,3,H,W]) → (feat [k,S,E] bf16,
    pos [k,S,2] i64)."""
    world, rank = _world(group)
    idx = [int(i) for i in idx]
    per = math.ceil(len(idx) / world)
    mine = idx[rank::world]
    S, E = frames.feat.shape[-2:]
    loc = torch.zeros((per, S * E * 2), dtype=torch.uint8, device=frames.feat.device)
    if mine:
        imgs = torch.cat([frames.img[i] for i in mine])
        feat, _ = encode(imgs)
        loc[:len(mine)] = feat.reshape(len(mine), S, E).contiguous().view(torch.uint8).reshape(
            len(mine), -1)
    allf = all_gather_rows(loc, len(idx), group)
    feats = allf.view(torch.bfloat16).reshape(len(idx), 1, S, E)
    gh, gw = frames.h // 16, frames.w // 16
    y = torch.arange(gh, device=frames.pos.device)
    x = torch.arange(gw, device=frames.pos.device)
    pos = torch.cartesian_prod(y, x).view(1, S, 2)
    for k, i in enumerate(idx):
        frames.feat[i] = feats[k]
        frames.pos[i] = pos


def keyframe_record_bytes(n):
    """Bytes of one packed keyframe record: X_canon f32 [n,3], C f32 [n], N i32, N_updates i32,
    T_WC f32 [8].  N and N_updates are separate counters (frame.py update_pointmap: only
    the weighted_pointmap mode keeps them equal)."""
    return (3 * n + n) * 4 + 8 + 32


def all_gather_keyframes(frames, idx, owner, group=None):
    """Keyframes idx[k] are authoritative on rank owner[k] (the rank that tracked / fused /
    appended them); one all-gather of padded per-rank buffers writes every keyframe's
    X_canon, C, N and T_WC into every rank's store (and the host count mirrors).  Ranks own
    any subset; the ownership map must be the same on every rank."""
    world, rank = _world(group)
    idx, owner = [int(i) for i in idx], [int(o) for o in owner]
    if world == 1 or not idx:
        return
    n = frames.h * frames.w
    rb = keyframe_record_bytes(n)
    if len(set(owner)) == 1:
        # one authoritative rank (the tracking rank): a broadcast, no padded slots
        src = owner[0]
        buf = torch.empty((len(idx), rb), dtype=torch.uint8, device=frames.X.device)
        if rank == src:
            for slot, k in enumerate(idx):
                _pack_keyframe(frames, k, buf[slot], n)
        dist.broadcast(buf, src, group=group)
        _unpack_keyframes(frames, idx, [buf[s] for s in range(len(idx))], n)
        return
    per = max(sum(1 for o in owner if o == r) for r in range(world))
    loc = torch.zeros((max(per, 1), rb), dtype=torch.uint8, device=frames.X.device)
    mine = [k for k, o in zip(idx, owner) if o == rank]
    for slot, k in enumerate(mine):
        _pack_keyframe(frames, k, loc[slot], n)
    gathered = [torch.empty_like(loc) for _ in range(world)]
    dist.all_gather(gathered, loc, group=group)
    slots = [0] * world
    recs = []
    for o in owner:
        recs.append(gathered[o][slots[o]])
        slots[o] += 1
    _unpack_keyframes(frames, idx, recs, n)


def _pack_keyframe(frames, k, rec, n):
    rec[:16 * n] = torch.cat((frames.X[k].reshape(-1), frames.C[k].reshape(-1))).view(torch.uint8)
    rec[16 * n:16 * n + 4] = frames.N[k:k + 1].to(torch.int32).view(torch.uint8)
    rec[16 * n + 4:16 * n + 8] = frames.N_updates[k:k + 1].to(torch.int32).view(torch.uint8)
    rec[16 * n + 8:] = frames.T_WC[k].reshape(8).contiguous().view(torch.uint8)


def _unpack_keyframes(frames, idx, recs, n):
    counts = {}
    for k, rec in zip(idx, recs):
        xc = rec[:16 * n].view(torch.float32)
        frames.X[k].copy_(xc[:3 * n].reshape(n, 3))
        frames.C[k].copy_(xc[3 * n:].reshape(n, 1))
        cnt = rec[16 * n:16 * n + 8].view(torch.int32)      # (N, N_updates)
        frames.N[k] = cnt[0]
        frames.N_updates[k] = cnt[1]
        frames.T_WC[k].copy_(rec[16 * n + 8:].view(torch.float32).reshape(1, 8))
        counts[k] = cnt
    # host mirrors of the counts (one device read for all of them)
    if counts:
        ks = list(counts)
        vals = torch.stack([counts[k] for k in ks]).tolist()
        for k, (vn, vu) in zip(ks, vals):
            frames._h_N[k], frames._h_Nu[k] = int(vn), int(vu)


def _is_gloo(group=None):
    return dist.get_backend(group) == "gloo"


def _all_gather_fixed(t, group=None):
    """all_gather of one equal-shape tensor per rank → [world, *t.shape] on t's device.
    gloo (the CPU test backend) stages device tensors through the host."""
    world, _ = _world(group)
    stage = t.is_cuda and _is_gloo(group)
    src = t.cpu() if stage else t.contiguous()
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src, group=group)
    r = torch.stack(out)
    return r.to(t.device) if stage else r


class ShardedFactorGraph(FactorGraph):
    """FactorGraph whose per-edge work is split across the ranks.

    Edge e of an add_factors call is matched on rank e % world, and its records (idx,
    valid, Q of both directions: 18 B/pixel) STAY on that rank: only the two per-edge
    match fractions (16 B) are all-gathered for the acceptance rule, which then runs
    identically everywhere.  ii / jj / owner are global on every rank; idx_ii2jj,
    idx_jj2ii, valid_match_*, Q_* hold this rank's accepted edges only, in global edge
    order.  solve_GN_* shards the Gauss-Newton edge pass the same way: each rank
    accumulates its own two-way edges' 35 per-edge sums (m3s_gn_*_edge_pass), one
    all-gather per iteration of E x 35 f64 (35 KB at E = 128) puts them in edge order on
    every rank, and every rank runs the same fp64 solve + retraction — the poses equal
    the unsharded solve's bit for bit (same per-edge sums, same assembly order)."""

    def __init__(self, *args, group=None, **kw):
        super().__init__(*args, **kw)
        self.group = group
        self.owner = torch.as_tensor([], dtype=torch.int32, device=self.device)

    def _match_local(self, ii, jj):
        return FactorGraph.match_edges(self, ii, jj)

    def match_edges(self, ii, jj):
        """Every edge's records on every rank (one all-gather of the packed records) — the
        base-class contract; add_factors below keeps records where they were computed."""
        world, rank = _world(self.group)
        if world == 1:
            return self._match_local(ii, jj)
        ii, jj = [int(i) for i in ii], [int(j) for j in jj]
        E = len(ii)
        n = self.frames.h * self.frames.w
        per = math.ceil(E / world)
        mine = list(range(rank, E, world))
        loc = torch.zeros((per, record_bytes(n)), dtype=torch.uint8, device=self.device)
        if mine:
            r = self._match_local([ii[e] for e in mine], [jj[e] for e in mine])
            loc[:len(mine)] = pack_edges(r, n)
        return unpack_edges(all_gather_rows(loc, E, self.group), n)

    def add_factors(self, ii, jj, min_match_frac, is_reloc=False):
        """global_opt2.py:35-107 with the records kept on the rank that matched them."""
        world, rank = _world(self.group)
        if world == 1:
            n0 = self.ii.numel()
            added = super().add_factors(ii, jj, min_match_frac, is_reloc)
            self.owner = torch.cat([self.owner, torch.zeros(self.ii.numel() - n0,
                                                            dtype=torch.int32, device=self.device)])
            return added
        ii, jj = [int(i) for i in ii], [int(j) for j in jj]
        E = len(ii)
        mine = list(range(rank, E, world))
        per = math.ceil(E / world)
        fr = torch.zeros((per, 2), dtype=torch.float64, device=self.device)
        r = None
        if mine:
            r = self._match_local([ii[e] for e in mine], [jj[e] for e in mine])
            vj = r["valid_match_j"] & (r["Qj"] > self.cfg["Q_conf"])
            vi = r["valid_match_i"] & (r["Qi"] > self.cfg["Q_conf"])
            fr[:len(mine), 0] = vj.sum(dim=(1, 2)).double() / (vj.shape[1] * vj.shape[2])
            fr[:len(mine), 1] = vi.sum(dim=(1, 2)).double() / (vi.shape[1] * vi.shape[2])
        frac = all_gather_rows(fr, E, self.group).float()   # edge order (round-robin slots)
        ii_t = torch.as_tensor(ii, device=self.device)
        jj_t = torch.as_tensor(jj, device=self.device)
        invalid = torch.minimum(frac[:, 0], frac[:, 1]) < min_match_frac
        invalid = (~(ii_t == (jj_t - 1))) & invalid
        if is_reloc and bool(invalid.any()):
            return False
        ok = ~invalid
        owner = torch.arange(E, device=self.device, dtype=torch.int32) % world
        self.ii = torch.cat([self.ii, ii_t[ok]])
        self.jj = torch.cat([self.jj, jj_t[ok]])
        self.owner = torch.cat([self.owner, owner[ok]])
        if r is not None:
            okm = ok[torch.as_tensor(mine, device=self.device)]
            self.idx_ii2jj = torch.cat([self.idx_ii2jj, r["idx_i2j"][okm]])
            self.idx_jj2ii = torch.cat([self.idx_jj2ii, r["idx_j2i"][okm]])
            self.valid_match_j = torch.cat([self.valid_match_j, r["valid_match_j"][okm]])
            self.valid_match_i = torch.cat([self.valid_match_i, r["valid_match_i"][okm]])
            self.Q_ii2jj = torch.cat([self.Q_ii2jj, r["Qj"][okm]])
            self.Q_jj2ii = torch.cat([self.Q_jj2ii, r["Qi"][okm]])
        return bool(ok.sum() > 0)

    def prep_two_way_edges(self):
        """The base class pairs ii / jj with idx / valid / Q row by row; with world > 1 ii / jj
        are global while those records are this rank's own edges, so the pairing would be
        silently misaligned: only the sharded solver (_solve_sharded) may read them."""
        if _world(self.group)[0] > 1:
            raise RuntimeError("ShardedFactorGraph.prep_two_way_edges: with world > 1 the match "
                               "records are rank-local (use solve_GN_* / local_edge_ids)")
        return super().prep_two_way_edges()

    def local_valid_fraction(self):
        """(valid match pixels, pixels) over this rank's accepted edges, both directions."""
        v = torch.cat((self.valid_match_j, self.valid_match_i))
        return float(v.sum()), float(v.numel())

    def valid_match_fraction(self):
        """Valid-match fraction over ALL accepted edges of the graph (every rank's records,
        summed with one all-reduce when world > 1)."""
        num, den = self.local_valid_fraction()
        world, _ = _world(self.group)
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([num, den], dtype=torch.float64,
                             device="cpu" if _is_gloo(self.group) else self.device)
            dist.all_reduce(t, group=self.group)
            num, den = float(t[0]), float(t[1])
        return num / den if den else 0.0

    def local_edge_ids(self):
        """Global two-way edge ids of this rank's rows (prep_two_way_edges order: the E
        i→j edges, then the same E as j→i)."""
        _, rank = _world(self.group)
        E = self.ii.numel()
        loc = torch.nonzero(self.owner == rank).flatten().to(torch.int32)
        return torch.cat([loc, loc + E])

    def solve_GN_rays(self):
        if _world(self.group)[0] == 1:
            return super().solve_GN_rays()
        self._solve_sharded("rays")

    def solve_GN_calib(self):
        if _world(self.group)[0] == 1:
            return super().solve_GN_calib()
        self._solve_sharded("calib")

    def _solve_sharded(self, mode):
        """global_opt2.py:129-221 with the GN edge pass sharded (class doc)."""
        import ctypes
        from . import _lib
        from .global_opt import constrain_points_to_ray
        world, rank = _world(self.group)
        c = self.cfg
        pin = c["pin"]
        uniq = self.get_unique_kf_idx()
        if uniq.numel() <= pin:
            return
        Xs, T_WCs, Cs = self.get_poses_points(uniq)
        if mode == "calib":
            Xs = constrain_points_to_ray((self.frames.h, self.frames.w), Xs, self.K)
        Xs, Cs = Xs.contiguous(), Cs.contiguous()
        ii = torch.cat((self.ii, self.jj)).contiguous()
        jj = torch.cat((self.jj, self.ii)).contiguous()
        # the edge → rank map on the host once (one small copy) — the slab layout below is
        # host arithmetic, not a device bincount / nonzero per rank (each a sync)
        owner_h = self.owner.cpu().long()
        E = self.ii.numel()
        mine = torch.nonzero(owner_h == rank).flatten()
        ids = torch.cat([mine, mine + E]).to(torch.int32).to(self.device).contiguous()
        idx = torch.cat((self.idx_ii2jj, self.idx_jj2ii)).contiguous()
        valid = torch.cat((self.valid_match_j, self.valid_match_i)).contiguous()
        Q = torch.cat((self.Q_ii2jj, self.Q_jj2ii)).contiguous()
        pose = T_WCs[:, 0, :].contiguous()
        P, N = Xs.shape[0], Xs.shape[1]
        E2, El = ii.numel(), ids.numel()
        lib, ptr, dev = _lib.load(), _lib.ptr, self.device
        s = _lib.stream(dev)
        ws = torch.empty(int(lib.m3s_gn_sharded_workspace_bytes(P, E2, El, N)), dtype=torch.uint8,
                         device=dev)
        dx = torch.zeros((max(P - 1, 1), 7), dtype=torch.float32, device=dev)
        # the per-edge rows all-gather as equal-size padded slabs; where each rank's rows go
        counts = torch.bincount(owner_h, minlength=world).tolist()
        pad = max(1, 2 * max(counts))
        G_loc = torch.zeros((pad, 35), dtype=torch.float64, device=dev)
        G_all = torch.zeros((E2, 35), dtype=torch.float64, device=dev) if world > 1 else None
        slot = []                                  # gathered row → global two-way edge id
        for r_ in range(world):
            loc = torch.nonzero(owner_h == r_).flatten()
            slot.append(torch.cat([loc, loc + E, torch.full((pad - 2 * loc.numel(),), -1,
                                                           dtype=loc.dtype)]))
        slot = torch.cat(slot)
        if world == 1:  # slot is the identity over the 2E two-way rows (pad == 2E)
            assert pad == E2 and torch.equal(slot, torch.arange(E2))
        take_h = torch.nonzero(slot >= 0).flatten()  # index lists, built once: no per-
        take = take_h.to(dev)                         # iteration mask (a host sync)
        dst = slot.index_select(0, take_h).to(dev)
        _lib.check(lib.m3s_gn_sharded_begin(ptr(ii), ptr(jj), P, N, E2, El, ptr(dx), ptr(ws), s),
                   "gn_sharded_begin")
        loop_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        loop_ev[0].record()                       # the iterations alone (gn_loop_ms)
        for _ in range(int(c["max_iters"])):
            if mode == "rays":
                st = lib.m3s_gn_rays_edge_pass(
                    ptr(pose), ptr(Xs), ptr(Cs), ptr(ids), ptr(idx), ptr(valid), ptr(Q), P, N,
                    E2, El, float(c["sigma_ray"]), float(c["sigma_dist"]), float(c["C_conf"]),
                    float(c["Q_conf"]), ptr(G_loc), ptr(ws), s)
            else:
                h, w = self.frames.h, self.frames.w
                st = lib.m3s_gn_calib_edge_pass(
                    ptr(pose), ptr(Xs), ptr(Cs), ptr(self.K.contiguous()), ptr(ids), ptr(idx),
                    ptr(valid), ptr(Q), P, N, E2, El, h, w, int(c["pixel_border"]),
                    float(c["depth_eps"]), float(c["sigma_pixel"]), float(c["sigma_depth"]),
                    float(c["C_conf"]), float(c["Q_conf"]), ptr(G_loc), ptr(ws), s)
            _lib.check(st, "gn_edge_pass")
            if world > 1:
                gathered = _all_gather_fixed(G_loc, self.group).reshape(world * pad, 35)
                G_all.index_copy_(0, dst, gathered.index_select(0, take))
                G_use = G_all
            else:  # one rank holds every edge: its slab is already in two-way edge order
                G_use = G_loc
            _lib.check(lib.m3s_gn_solve_step(ptr(pose), ptr(G_use), P, N, E2, El,
                                             float(c["delta_norm"]), ptr(dx), ptr(ws), s),
                       "gn_solve_step")
        loop_ev[1].record()
        hs, it = ctypes.c_int(0), ctypes.c_int(0)
        _lib.check(lib.m3s_gn_sharded_status(ptr(ws), P, ctypes.byref(hs), ctypes.byref(it), s),
                   "gn_sharded_status")
        if hs.value == -1:
            raise RuntimeError("gauss_newton (sharded): the number of unique keyframes in ii/jj "
                               "must equal Xs.size(0)")
        self.gn_iterations = it.value
        self.gn_loop_ms = loop_ev[0].elapsed_time(loop_ev[1])   # status call synchronised
        T_WCs[:, 0, :] = pose
        self.frames.update_T_WCs(T_WCs[pin:], uniq[pin:])
