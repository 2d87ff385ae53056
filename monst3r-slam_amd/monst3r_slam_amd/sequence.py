"""The C3 workload (BASELINE configs[2]): the main loop's TRACKING branch
(main_monster_slam.py:247-332 with FrameTracker2.track, tracker2.py:70-270) over a
synthetic 384x512 sequence, every frame a new image, the keyframe replaced whenever the
tracker asks for a new one — all of it replayable from captured HIP graphs.

Scene: a textured box room with box-shaped furniture (never a single
plane in view: a planar view leaves the ray-only Sim3 residual nearly degenerate along the
viewing direction) seen by a pinhole camera (fx = fy = 400,
cx = w/2, cy = h/2) moving on a smooth periodic trajectory (yaw ±0.6 rad, translation,
pitch/roll wobble; period 200 frames).  Per frame f, staged in HBM before the timed region:
  Xcam[f]    the frame's own pointmap (ray-cast depth, x (1 + 1e-3 N(0,1)) noise)
  D16[f]     24-d unit descriptors of the world point (smooth random texture field), f16
  C / Q      1 + exp(N(1, .5)) per pixel (own view, other view)
  img[f]     the rendered texture colours in [-1, 1] (what the encoder sees)
  T_gt[f]    camera-to-world Sim3 (scale 1)
Trained weights are absent and random weights regress no geometry, so after the ViT pair
inference has run on img[f] (its real cost, in stream order) m3s_seq_pair_outputs
overwrites its X / C / D16 / Q with what a perfect network would regress for (frame t,
keyframe j): Xii = Xcam[t], Xji = T_t^-1 T_j Xcam[j], D = (D16[t], D16[j]).  Matching, the
pose solve, keyframe fusion and the keyframe decisions then run on real geometry, frame
after frame, with the previous frame's matches and pose as the next frame's seed.
"""
from __future__ import annotations

import math

import numpy as np

import torch

from . import _lib
from . import synthetic as syn

LOG_INTS = 8   # m3s_seq_advance log row: iters, new_kf, lost, kf_frame, chol_fail, recovered


def trajectory(n_frames, period=200, yaw=0.6):
    """GT camera-to-world Sim3 poses [n, 8] (t, q xyzw, s = 1); frame 0 is the identity."""
    out = np.zeros((n_frames, 8), np.float32)
    for t in range(n_frames):
        ph = 2.0 * math.pi * t / period
        c = np.array([0.6 * math.sin(ph), 0.1 * math.sin(2 * ph), 0.4 * (1.0 - math.cos(ph))])
        qy = syn.quat_from_axis_angle([0, 1, 0], yaw * math.sin(ph))
        qx = syn.quat_from_axis_angle([1, 0, 0], 0.08 * math.sin(3 * ph))
        qz = syn.quat_from_axis_angle([0, 0, 1], 0.03 * math.sin(2 * ph))
        T = syn.sim3_mul(syn.sim3_mul(np.concatenate([[0, 0, 0], qy, [1.0]]),
                                      np.concatenate([[0, 0, 0], qx, [1.0]])),
                         np.concatenate([[0, 0, 0], qz, [1.0]]))
        T[:3] = c
        out[t] = T
    return out


def _quat_to_rot_t(q):
    x, y, z, w = q.unbind(-1)
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


class _Texture:
    def __init__(self, device, dim=24, seed=7, freq=25.0):
        g = torch.Generator().manual_seed(seed)
        self.freqs = (torch.randn(2 * dim, 3, generator=g) * freq).to(device)
        self.phases = (torch.rand(2 * dim, generator=g) * 2 * math.pi).to(device)
        self.R = torch.randn(2 * dim, dim, generator=g).to(device)
        self.cf = (torch.randn(3, 3, generator=g) * 6.0).to(device)
        self.cp = (torch.rand(3, generator=g) * 2 * math.pi).to(device)

    def desc(self, P):
        D = torch.sin(P @ self.freqs.T + self.phases) @ self.R
        return D / D.norm(dim=-1, keepdim=True)

    def colour(self, P):
        return torch.sin(P @ self.cf.T + self.cp)          # [-1, 1]


class SyntheticSequence:
    """The staged sequence (see module doc).  Tensors on `device`, frame-major."""

    ROOM_LO = (-3.0, -1.6, -3.5)
    ROOM_HI = (3.0, 1.6, 5.0)
    # furniture (lo, hi): clear of the camera path (|x| <= 0.6, 0 <= z <= 0.8)
    BOXES = (((1.2, -1.6, 2.5), (2.0, 0.2, 3.3)), ((-2.2, -1.6, 1.5), (-1.2, -0.2, 2.6)),
             ((-0.8, -1.6, 3.2), (0.4, -0.9, 4.2)), ((-2.9, -1.6, -1.0), (-2.3, 1.6, 0.0)),
             ((2.2, -0.5, -0.5), (2.9, 1.2, 1.0)), ((-0.3, 0.6, 4.2), (0.9, 1.6, 5.0)),
             ((-2.0, 0.4, 3.6), (-1.1, 1.3, 4.4)), ((1.1, -1.6, -2.8), (2.4, -0.4, -1.8)))

    def __init__(self, n_frames, h=384, w=512, device="cpu", seed=0, period=200, noise=1e-3,
                 lost_frames=(), tex_freq=25.0):
        dev = torch.device(device)
        self.n_frames, self.h, self.w, self.n = n_frames, h, w, h * w
        self.device, self.period = dev, period
        # fx = fy = 400 at 512 wide; scaled with the width for smaller runs
        self.K = syn.intrinsics(h, w)
        self.K[0, 0] = self.K[1, 1] = 400.0 * w / 512.0
        T = trajectory(n_frames, period)
        self.T_gt_np = T
        self.T_gt = torch.from_numpy(T).to(dev)
        n = self.n
        self.Xcam = torch.empty((n_frames, n, 3), dtype=torch.float32, device=dev)
        self.D16 = torch.empty((n_frames, n, 24), dtype=torch.float16, device=dev)
        self.C_own = torch.empty((n_frames, n), dtype=torch.float32, device=dev)
        self.C_other = torch.empty_like(self.C_own)
        self.Q_own = torch.empty_like(self.C_own)
        self.Q_other = torch.empty_like(self.C_own)
        self.img = torch.empty((n_frames, 1, 3, h, w), dtype=torch.float32, device=dev)
        tex = _Texture(dev, freq=tex_freq)
        yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32, device=dev),
                                torch.arange(w, dtype=torch.float32, device=dev), indexing="ij")
        K = self.K
        dc = torch.stack([(xx - float(K[0, 2])) / float(K[0, 0]),
                          (yy - float(K[1, 2])) / float(K[1, 1]), torch.ones_like(xx)], -1)
        dc = dc.reshape(n, 3)
        lo = torch.tensor(self.ROOM_LO, device=dev)
        hi = torch.tensor(self.ROOM_HI, device=dev)
        for f in range(n_frames):
            g = torch.Generator(device=dev).manual_seed(seed * 100003 + f)
            Tf = self.T_gt[f]
            R = _quat_to_rot_t(Tf[3:7])
            c = Tf[:3]
            dw = dc @ R.T
            bound = torch.where(dw > 0, hi, lo)
            tax = (bound - c) / torch.where(dw == 0, torch.full_like(dw, 1e-30), dw)
            tax = torch.where(tax > 0, tax, torch.full_like(tax, float("inf")))
            thit = tax.min(-1).values
            for blo, bhi in self.BOXES:          # slab test, entry distance if in front
                blo = torch.tensor(blo, device=dev)
                bhi = torch.tensor(bhi, device=dev)
                inv = 1.0 / torch.where(dw == 0, torch.full_like(dw, 1e-30), dw)
                t0 = (blo - c) * inv
                t1 = (bhi - c) * inv
                tn = torch.minimum(t0, t1).max(-1).values
                tf = torch.maximum(t0, t1).min(-1).values
                hit = (tn <= tf) & (tn > 0)
                thit = torch.where(hit & (tn < thit), tn, thit)
            Xw = c + thit[:, None] * dw
            Xc = thit[:, None] * dc
            Xc = Xc * (1.0 + noise * torch.randn(n, 1, device=dev, generator=g))
            self.Xcam[f] = Xc
            self.D16[f] = tex.desc(Xw).half()
            for buf in (self.C_own, self.C_other, self.Q_own, self.Q_other):
                buf[f] = 1.0 + torch.exp(1.0 + 0.5 * torch.randn(n, device=dev, generator=g))
            self.img[f, 0] = tex.colour(Xw).T.reshape(3, h, w)
        for f in lost_frames:
            # an unusable frame (every Qk <= Q_conf → match_frac 0 → lost, tracker2.py:211-213)
            self.Q_own[f] = 1.2
            self.Q_other[f] = 1.2

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (
            self.Xcam, self.D16, self.C_own, self.C_other, self.Q_own, self.Q_other, self.img))


class SequenceLoop:
    """The main loop's TRACKING branch over a SyntheticSequence on the device:
    step() = (prefetched) encoder of the next image, pair inference vs the current keyframe,
    the stand-in pair outputs, FrameTracker2.track glue + pose solve, then m3s_seq_advance
    (log, next frame's initial pose, keyframe replacement, idx_f2k reset).  No host
    synchronisation: capture two steps (feature parities 0 / 1) and replay them alternately."""

    def __init__(self, tracker, seq: SyntheticSequence, pipe=None):
        self.tr, self.seq, self.pipe = tracker, seq, pipe
        dev = seq.device
        self.dev = dev
        self.frame = torch.zeros(1, dtype=torch.int32, device=dev)
        self.kf_frame = torch.zeros(1, dtype=torch.int32, device=dev)
        self.T_prev = torch.zeros(8, dtype=torch.float32, device=dev)
        self.log_i = torch.zeros((seq.n_frames, LOG_INTS), dtype=torch.int32, device=dev)
        self.log_T = torch.zeros((seq.n_frames, 8), dtype=torch.float32, device=dev)
        self.img_cur = torch.empty((1, 3, seq.h, seq.w), dtype=torch.float32, device=dev)
        g = pipe.group if pipe is not None else 1
        self.img_next = torch.empty((g, 3, seq.h, seq.w), dtype=torch.float32, device=dev)
        # pipelined: the side stream's gather reads the device frame counter that advance()
        # rewrites on the main stream; this event orders advance() after the gather
        self._gathered = torch.cuda.Event() if dev.type == "cuda" else None

    # ---- INIT (main_monster_slam.py:279-290) ----
    def reset(self, first=0, parity=0):
        """Keyframe 0 = frame `first` at the identity pose (its mono pointmap: the stand-in's
        own-view geometry), idx_f2k identity, the next frame to track = first + 1; with a
        pipeline, that frame's features are encoded into buffer `parity`."""
        s, tr = self.seq, self.tr
        T0 = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1], dtype=torch.float32, device=self.dev)
        X = s.Xcam[first].clone()
        C = s.C_own[first].reshape(-1, 1).clone()
        if tr.model is not None:
            feat, _ = tr.model.encode(s.img[first])
            feat = feat.clone()
        else:
            feat = torch.zeros(16, dtype=torch.uint8, device=self.dev)
        if tr.kf is None or tr.kf.X_canon.shape != X.shape:
            tr.add_keyframe(s.img[first], T0, X=X, C=C, feat=feat)
        else:
            tr.kf.X_canon.copy_(X)
            tr.kf.C.copy_(C)
            tr.kf.N.fill_(1.0)
            tr.kf.T_WC.copy_(T0)
            tr.kf.feat.copy_(feat.reshape(tr.kf.feat.shape))
            # in place: captured graphs hold the buffer's address
            tr.idx_f2k.copy_(torch.arange(X.shape[0], device=self.dev)[None])
        self.frame.fill_(first + 1)
        self.kf_frame.fill_(first)
        self.T_prev.copy_(T0)
        self.log_i.zero_()
        self.log_T.zero_()
        if self.pipe is not None:
            g = self.pipe.group
            if parity % g:
                # prime() fills rows 0..g-1 of the group buffer (parity // g) % 2, and step
                # k tracks row k % g: a parity inside a group would track rows that part 0
                # of that group never embedded
                raise ValueError(f"reset: parity {parity} must be a multiple of the prefetch "
                                 f"group {g}")
            if first + g >= s.n_frames:
                raise ValueError("sequence too short for the prefetch group")
            self.pipe.prime(s.img[first + 1:first + 1 + g].reshape(g, 3, s.h, s.w), parity)

    def gather(self, dst, offset):
        s = self.seq
        lib = _lib.load()
        fb = s.img[0].numel() * 4
        _lib.check(lib.m3s_seq_gather(_lib.ptr(s.img), fb, _lib.ptr(self.frame), offset,
                                      s.n_frames, _lib.ptr(dst), _lib.stream(self.dev)),
                   "seq_gather")

    def pair_outputs(self, out):
        s = self.seq
        X, C, D16, Q = out["X"], out["C"], out["D16"], out["Q"]
        assert X.is_contiguous() and C.is_contiguous() and D16.is_contiguous() and \
            Q.is_contiguous(), "pair outputs must be contiguous [2,H,W,*]"
        assert X.shape == (2, s.h, s.w, 3) and D16.shape == (2, s.h, s.w, 24)
        P = _lib.ptr
        _lib.check(_lib.load().m3s_seq_pair_outputs(
            P(s.Xcam), P(s.C_own), P(s.C_other), P(s.Q_own), P(s.Q_other), P(s.D16), P(s.T_gt),
            P(self.frame), P(self.kf_frame), s.n_frames, s.n, P(X), P(C), P(D16), P(Q),
            _lib.stream(self.dev)), "seq_pair_outputs")

    def advance(self, res, out, feat_i):
        s, kf = self.seq, self.tr.kf
        flags = self.tr._glue["flags"] if self.tr._glue is not None else None
        if flags is None:
            raise RuntimeError("SequenceLoop needs the fused tracking glue (M3S_FUSED_GLUE=1)")
        fb = 0 if feat_i is None else feat_i.numel() * feat_i.element_size()
        if fb and kf.feat.numel() * kf.feat.element_size() != fb:
            raise RuntimeError("keyframe feature buffer size mismatch")
        P = _lib.ptr
        _lib.check(_lib.load().m3s_seq_advance(
            P(flags), P(res["info"]), P(res["T_WCf"]), P(out["X"]), P(out["C"]),
            P(feat_i) if fb else None, fb, s.n, P(kf.X_canon), P(kf.C), P(kf.N), P(kf.T_WC),
            P(kf.feat) if fb else None, P(self.tr.idx_f2k), P(self.T_prev), P(self.frame),
            P(self.kf_frame), P(self.log_i), P(self.log_T), s.n_frames, _lib.stream(self.dev)),
            "seq_advance")

    def step(self, k=0, split_heads=None):
        """One frame; k = the step index modulo the pipeline's period (feature-buffer slot).  res["idx_f2k"] is the
        tracker's persistent match buffer (the next frame's seed, written in place by the
        matcher): after a keyframe replacement advance() has already reset it to the
        identity, as tracker2.py:255-257 does before the next frame."""
        tr, m, pipe = self.tr, self.tr.model, self.pipe
        split = tr.split_heads if split_heads is None else split_heads
        main = torch.cuda.current_stream(self.dev)
        feat_i = None
        if m is not None:
            if pipe is not None:
                feat_i = pipe.slot(k)
                # group g: only part 0 of a group encode reads the images
                gathers = k % pipe.group == 0

                def prefetch():
                    pipe.side.wait_stream(main)
                    with torch.cuda.stream(pipe.side):
                        if gathers:   # group g: the frames g .. 2g-1 after the tracked one
                            for j in range(pipe.group):
                                self.gather(self.img_next[j:j + 1], pipe.group + j if
                                            pipe.group > 1 else 1)
                            self._gathered.record(pipe.side)
                        pipe.encode_side(self.img_next, k)
                # (issued before the pair: the encoder fills the decoder phase.  Started once
                # the decoders are issued instead, into the head phase's idle CUs: 196 vs
                # 231.5 frames/s, round 5 — the head phase cannot absorb it)
                prefetch()
                out = m.pair(self.img_cur, feat_j=tr.kf.feat, feat_i=feat_i, split_heads=split)
            else:
                self.gather(self.img_cur, 0)
                out = m.pair(self.img_cur, feat_j=tr.kf.feat, split_heads=split)
                feat_i = out["feat_i"]
        else:
            out = self._outputs()
        self.pair_outputs(out)
        res = tr.track_outputs(out, self.T_prev)
        if pipe is not None and m is not None and gathers:
            main.wait_event(self._gathered)   # the gather read `frame` before advance rewrites it
        self.advance(res, out, feat_i if m is not None else None)
        if m is not None:
            m.join()
            if pipe is not None:
                main.wait_stream(pipe.side)
        res["pair"] = out
        return res

    def _outputs(self):
        """Pair-output buffers when there is no model (glue-only runs)."""
        if not hasattr(self, "_out"):
            s, dev = self.seq, self.dev
            self._out = dict(X=torch.empty((2, s.h, s.w, 3), device=dev),
                             C=torch.empty((2, s.h, s.w), device=dev),
                             D16=torch.empty((2, s.h, s.w, 24), dtype=torch.float16, device=dev),
                             Q=torch.empty((2, s.h, s.w), device=dev))
        return self._out

    def summary(self, first=0, count=None):
        """Host summary of the logged frames first+1 .. first+count (one sync)."""
        li = self.log_i.cpu().numpy()
        lt = self.log_T.cpu().numpy()
        a = first + 1
        b = self.seq.n_frames if count is None else min(self.seq.n_frames, a + count)
        li, lt = li[a:b], lt[a:b]
        iters = li[:, 0]
        hist = {int(k): int(v) for k, v in zip(*np.unique(iters, return_counts=True))}
        return dict(frames=int(b - a), keyframes_added=int(li[:, 1].sum()),
                    keyframes_total=int(li[:, 1].sum()) + 1, lost=int(li[:, 2].sum()),
                    cholesky_failures=int(li[:, 4].sum()), recovered=int((li[:, 5] > 0).sum()),
                    gn_iterations_hist=hist, gn_iterations_mean=float(iters.mean()),
                    T_WC=lt, log=li)


def ate_vs_gt(T_est, T_gt):
    """Sim3-aligned ATE rmse (evaluate.ate's Umeyama on the translations)."""
    from . import evaluate as E
    return E.ate_arrays(np.asarray(T_est)[:, :3], np.asarray(T_gt)[:, :3])
