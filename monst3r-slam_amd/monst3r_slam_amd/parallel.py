"""Keyframe-graph work sharded over the GPUs of one node.

Tracking is sequential (frame t needs the pose and matches of t-1), so it runs as
independent replicas.  The keyframe graph is data-parallel: every candidate edge's
symmetric inference (4 directed decodes + 8 heads) and its two matchings are
independent, and so is every keyframe's encoder pass.  One process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI on the MI355X node, "gloo" in the
CPU tests):

  shard_keyframe_features  keyframes encoded round-robin across ranks, features
                           all-gathered (1.5 MB bf16 per keyframe at 384x512)
  ShardedFactorGraph       FactorGraph whose match_edges runs the rank's round-robin share
                           of the edges and all-gathers one packed record per edge
                           (idx i32 x2, valid u8 x2, Q f32 x2 = 18 B/pixel, 3.5 MB/edge);
                           the acceptance rule and the GN solve then run identically on
                           every rank (the GN system is tiny; replicating it avoids a
                           broadcast of the poses).
  all_gather_keyframes     the keyframe pointmaps (X_canon, C, N, T_WC) each rank is
                           authoritative for — the tracking rank's fused keyframes, new
                           keyframes — all-gathered into every rank's keyframe store before
                           the backend reads them (3.1 MB per keyframe at 384x512), so the
                           replicated GN sees the same pointmaps everywhere
Each all-gather moves ceil(E/world) records per rank in ONE collective (padded), i.e.
world-1 of every world records cross xGMI once — no per-edge messages.
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


class ShardedFactorGraph(FactorGraph):
    """FactorGraph whose per-edge inference + matching is split across the ranks."""

    def __init__(self, *args, group=None, **kw):
        super().__init__(*args, **kw)
        self.group = group

    def _match_local(self, ii, jj):
        return FactorGraph.match_edges(self, ii, jj)

    def match_edges(self, ii, jj):
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
