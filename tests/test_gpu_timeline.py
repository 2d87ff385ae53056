"""GPU: the step timeline behind bench.py's roofline (m3s_timeline_set / _count / _meta,
include/monst3r_slam_amd.h): every GEMM / attention launch issued while it is armed takes
one slot, records its kind (1 GEMM, 2 attention, 3 implicit-conv GEMM), algorithmic FLOPs
and dims, and its blocks stamp [earliest start, latest end] — checked on one pair inference
of the small model, eager and captured into a graph."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_timeline_records_every_launch(dev):
    from monst3r_slam_amd import _lib
    from monst3r_slam_amd import model as Mdl
    lib, P = _lib.load(), _lib.ptr
    m, _ = Mdl.build(dev, small=True)
    H, W = 96, 128
    g = torch.Generator(device=dev).manual_seed(3)
    img = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
    feat_k, _ = m.encode(img)
    feat_k = feat_k.clone()
    m.pair(img, feat_j=feat_k)          # allocate outside the timeline
    torch.cuda.synchronize()
    cap = 2048
    slot = torch.empty((cap, 132), dtype=torch.int64, device=dev)   # M3S_TL_SLOT u64 per slot
    buf = slot[:, :128].view(cap, 64, 2)
    buf[..., 0] = -1
    buf[..., 1] = 0
    # block log: one 8-u64 record per block {start, end, slot address, HW_ID | XCC_ID << 32,
    # GEMM phase marks}
    nlog = 1 << 16
    blog = torch.zeros((nlog, 8), dtype=torch.int64, device=dev)
    bcnt = torch.zeros(2, dtype=torch.int32, device=dev)
    slot[:, 128:] = 7                    # garbage headers: m3s_timeline_set zeroes them
    m.ops.record = []
    _lib.check(lib.m3s_timeline_set(P(buf), cap), "timeline_set")
    assert int(slot[:, 128:].abs().sum()) == 0
    slot[:, 128] = blog.data_ptr()
    slot[:, 129] = bcnt.data_ptr()
    slot[:, 130] = nlog
    try:
        m.pair(img, feat_j=feat_k)
        torch.cuda.synchronize()
        n = int(lib.m3s_timeline_count())
        kinds = np.zeros(cap, np.int32)
        flops = np.zeros(cap, np.float64)
        dims = np.zeros((cap, 4), np.int64)
        _lib.check(lib.m3s_timeline_meta(kinds.ctypes.data, flops.ctypes.data, dims.ctypes.data,
                                         cap), "timeline_meta")
    finally:
        lib.m3s_timeline_set(None, 0)
    rec, m.ops.record = m.ops.record, None
    assert 0 < n < cap
    k = kinds[:n]
    assert set(np.unique(k)) <= {1, 2, 3} and (k == 2).any() and (k == 3).any()
    # one GEMM slot per recorded GEMM descriptor, same FLOPs, conv kind for mode-1 launches
    gemm = np.flatnonzero(k != 2)
    assert len(gemm) == len(rec)
    np.testing.assert_allclose(flops[gemm], [r[1] for r in rec])
    assert [int(x) for x in k[gemm] == 3] == [int(r[0].mode != 0) for r in rec]
    for i, r in zip(gemm, rec):
        assert tuple(dims[i]) == (r[0].M, r[0].N, r[0].K, r[0].batch)
    # attention FLOPs = 4 Sq Sk 64 heads batch
    at = np.flatnonzero(k == 2)
    np.testing.assert_allclose(flops[at], 4.0 * dims[at, 0] * dims[at, 1] * 64 * dims[at, 2]
                               * dims[at, 3])
    # every launch stamped: a start (< UINT64_MAX) before its end
    tb = buf[:n].cpu().numpy()
    st = np.where(tb[..., 0] > 0, tb[..., 0], np.iinfo(np.int64).max).min(1)
    en = tb[..., 1].max(1)
    assert (en > 0).all() and (st < en).all()
    # the block log: every block of every launch recorded once, inside its launch's span,
    # on a CU the hardware ids name (XCC 0-7)
    nb = int(bcnt[0])
    assert 0 < nb <= nlog
    lg = blog[:nb].cpu().numpy()
    base = slot.data_ptr()
    sl = (lg[:, 2] - base) // (132 * 8)
    assert ((lg[:, 2] - base) % (132 * 8) == 0).all() and (sl >= 0).all() and (sl < n).all()
    assert (lg[:, 0] <= lg[:, 1]).all()
    assert (lg[:, 0] >= st[sl]).all() and (lg[:, 1] <= en[sl]).all()
    xcc = (lg[:, 3] >> 32) & 0xF
    assert xcc.max() <= 7
    assert set(np.unique(sl)) == set(range(n))      # no launch without a block record
    # GEMM blocks carry their phase marks in order: prologue issued <= first K-tile ready <=
    # K-loop done <= epilogue tile in LDS, inside the block's lifetime; attention blocks none
    kk = k[np.clip(sl, 0, n - 1)]
    gm = lg[kk != 2]
    # (a separate split-K reduce launch logs its blocks into its GEMM's slot, unmarked)
    gm = gm[(gm[:, 4:8] != 0).any(1)]
    assert set(np.unique(sl[kk != 2])) == set(np.unique((gm[:, 2] - base) // (132 * 8)))
    ph = gm[:, 4:8]
    assert (ph[:, :3] > 0).all()           # (split-K slices that are not the last skip mark 3)
    assert (gm[:, 0] <= ph[:, 0]).all() and (np.diff(ph[:, :3], axis=1) >= 0).all()
    full = ph[:, 3] > 0
    assert full.mean() > 0.5 and (ph[full, 3] >= ph[full, 2]).all()
    assert (ph[full, 3] <= gm[full, 1]).all()
    assert (lg[kk == 2][:, 4:8] == 0).all()

