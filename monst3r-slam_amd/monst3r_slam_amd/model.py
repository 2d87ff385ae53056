"""MonST3R + MASt3R pair inference on the MI355X kernels (C ABI, bf16 MFMA).

Mirrors the reference's model-level operator API used by the SLAM frontend:
  _encode_image (d3r/model.py:127-139)  → PairModel.encode
  _decoder      (d3r/model.py:171-190)  → both models x both sides in ONE batched pass
  _downstream_head + postprocess        → all four DPT heads batched; MASt3R catmlp tail
  monst3r_asymmetric_inference (mast3r_slam/monst3r_utils.py:255-297) → PairModel.pair
Design:
  * residual streams f32, GEMM operands bf16, MFMA f32 accumulation;
  * z = model*2 + side batches the two decoder sides and the two models (4 independent
    problems with their own weights) into every decoder GEMM / attention / LN launch,
    and the four DPT heads likewise — M = 768 tokens alone fills only ~1/2 of the CUs;
  * DPT on NHWC bf16 with implicit-GEMM 3x3 convs (ReLU prologue, bias + residual
    epilogue), ConvTranspose(k=s) as GEMM + scatter epilogue, the fusion block's 1x1
    out_conv applied BEFORE the x2 upsample (linear ops commute; bilinear weights sum to
    one) and the skip add fused into the upsample;
  * the final 1x1 conv (128→4) + reg_dense_depth/conf fused in one tail kernel; the
    MASt3R MLP tail fused with pixel_shuffle + desc normalisation, emitting f16
    descriptors for matching directly (== .half() of the f32 unit vectors).
Weights: seeded random (monst3r_slam_amd.weights) — no checkpoints offline.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from . import weights as Wt

BF16 = torch.bfloat16
F32 = torch.float32
U8 = torch.uint8
LN_EPS = 1e-6


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _Nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class Ops:
    """Thin, checked wrappers over the ViT C ABI on the current torch stream."""

    def __init__(self, dev):
        self.lib = _lib.load()
        self.dev = dev
        self.record = None  # list → (descriptor, flops, fp8) per GEMM launch (bench roofline)
        self.tile_default = None  # tile hint for launches issued without one (side chains)
        # f32 split-K / attention-split scratch and the split-K tile counters (zeroed once,
        # left zero by the kernels), one set per stream (the M = 768 GEMMs split K when
        # their grid cannot fill 256 CUs; concurrent streams must not share them)
        self._ws = {}
        self._cnt = {}

    @property
    def ws(self):
        sid = torch.cuda.current_stream(self.dev).cuda_stream
        w = self._ws.get(sid)
        if w is None:
            w = torch.empty(64 << 20, dtype=torch.uint8, device=self.dev)
            self._ws[sid] = w
        return w

    @property
    def counters(self):
        sid = torch.cuda.current_stream(self.dev).cuda_stream
        c = self._cnt.get(sid)
        if c is None:
            c = torch.zeros(1 << 16, dtype=torch.int32, device=self.dev)
            self._cnt[sid] = c
        return c

    def _s(self):
        return _lib.stream(self.dev)

    def gemm(self, A, B, C, M, N, K, batch=1, *, lda=None, ldb=None, ldc=None, sA=0, sB=0,
             sC=0, bias=None, sBias=0, R=None, ldr=None, sR=0, flags=0, conv=None, convt=None,
             rope=None, split_k=0, wmod=0, dpt=None, fp8=None, out_fp8=False, ln_stats=None,
             ln_fold=None, tile=None):
        """fp8 = (col_scale f32 [.., N], stride): A and B are OCP e4m3 bytes (torch
        float8_e4m3fn / uint8), the f32 accumulator is scaled per column; out_fp8: C is
        stored as e4m3.
        ln_stats = (C2 bf16, stats f32 [batch, M, N/128, 2]): this f32-out GEMM produces a
        LayerNorm input — also store its bf16 copy and per-128-column (mean, M2);
        (C2 uint8, stats, shift f32 [.., N], qscale f32 [..]): the copy is e4m3 of
        (C − shift)·qscale instead (the fp8 consumer's A operand).
        ln_fold = (stats, c1 f32, a_xor[, c3 f32]): A is the bf16 (or shifted e4m3) copy of a
        LayerNorm input and B a gamma-folded weight; the epilogue applies the normalisation
        (bias = c2); c3 = Σ_k shift[k] B[n][k] for the shifted e4m3 copy.
        tile = (tile configuration, split-K): the descriptor's tile_hint instead of the
        per-shape table (PairModel.encode(concurrent=True))."""
        if tile is None:
            tile = self.tile_default
        d = _lib.GemmDesc()
        d.A, d.lda, d.strideA = _p(A), lda if lda is not None else K, sA
        d.B, d.ldb, d.strideB = _p(B), ldb if ldb is not None else K, sB
        d.C, d.ldc, d.strideC = _p(C), ldc if ldc is not None else N, sC
        d.bias, d.strideBias = _p(bias), sBias
        d.R, d.ldr, d.strideR = _p(R), ldr if ldr is not None else N, sR
        d.M, d.N, d.K, d.batch, d.flags = M, N, K, batch, flags
        ws = self.ws
        d.workspace, d.workspace_bytes, d.split_k = _p(ws), ws.numel(), split_k
        cnt = self.counters
        d.tile_counters, d.tile_counters_len = _p(cnt), cnt.numel()
        d.weight_mod = wmod
        if tile is not None:
            d.tile_hint, d.split_k = int(tile[0]), int(tile[1])
        if fp8 is not None:
            d.flags |= _lib.IN_FP8
            d.col_scale, d.stride_col_scale = _p(fp8[0]), fp8[1]
        if out_fp8:
            d.flags |= _lib.EPI_OUT_FP8
        if dpt is not None:  # fused DPT tail: (W4 [h][4][128], b4 [h][4], pts, conf, conf_min)
            d.flags |= _lib.EPI_DPT_OUT
            d.dpt_w4, d.dpt_b4, d.dpt_pts, d.dpt_conf = (_p(t) for t in dpt[:4])
            d.dpt_conf_min = float(dpt[4])
        if bias is not None:
            d.flags |= _lib.EPI_BIAS
        if conv is not None:
            d.mode = 1
            d.Hin, d.Win, d.Cin, d.Hout, d.Wout, d.stride = conv
        if convt is not None:
            d.flags |= _lib.EPI_CONVT
            d.ct_s, d.ct_cout, d.ct_gw = convt
        if rope is not None:  # (cos/sin table, rotated columns, tokens per image)
            d.flags |= _lib.EPI_ROPE
            d.rope_table, d.rope_cols, d.rope_tokens = _p(rope[0]), rope[1], rope[2]
        if ln_stats is not None:
            d.flags |= _lib.EPI_LN_STATS
            d.C2, d.stats = _p(ln_stats[0]), _p(ln_stats[1])
            if len(ln_stats) > 2 and ln_stats[2] is not None:
                d.ln_shift, d.ln_qscale = _p(ln_stats[2]), _p(ln_stats[3])
        if ln_fold is not None:
            d.flags |= _lib.EPI_LN_FOLD
            d.stats, d.ln_c1, d.a_batch_xor = _p(ln_fold[0]), _p(ln_fold[1]), ln_fold[2]
            d.stats_groups, d.ln_eps = K // 128, LN_EPS
            if len(ln_fold) > 3 and ln_fold[3] is not None:
                d.ln_c3 = _p(ln_fold[3])
        if self.record is not None:  # (descriptor copy, flops, fp8) for the bench replay
            dc = _lib.GemmDesc()
            ctypes.memmove(ctypes.byref(dc), ctypes.byref(d), ctypes.sizeof(d))
            self.record.append((dc, 2.0 * M * N * K * batch, fp8 is not None))
        _lib.check(self.lib.m3s_vit_gemm(ctypes.byref(d), self._s()), "vit_gemm")

    def replay_gemm(self, desc):
        """Re-issue a recorded GEMM descriptor on the current stream (bench roofline)."""
        _lib.check(self.lib.m3s_vit_gemm(ctypes.byref(desc), self._s()), "vit_gemm")

    def ln(self, x, g, b, y, rows, dim, batch=1, sx=0, sy=0, sp=0, y_f32=False, xor=0, pmod=0):
        """y dtype picks the output: bf16, f32 (or y_f32) or uint8/float8_e4m3fn (e4m3)."""
        yt = 1 if (y_f32 or y.dtype == F32) else 2 if y.element_size() == 1 else 0
        _lib.check(self.lib.m3s_vit_layernorm(
            _p(x), int(x.dtype == BF16), _p(g), _p(b), _p(y), yt, rows, dim, LN_EPS,
            batch, sx, sy, sp, pmod, xor, self._s()), "vit_layernorm")

    def ln_dual(self, x, g, b, y, g2, b2, y2, rows, dim, batch, sx, sy, sp, pmod=0):
        _lib.check(self.lib.m3s_vit_layernorm_dual(
            _p(x), _p(g), _p(b), _p(y), _p(g2), _p(b2), _p(y2), int(y.element_size() == 1), rows,
            dim, LN_EPS, batch, sx, sy,
            sp, pmod, self._s()), "vit_layernorm_dual")

    def rope(self, t, ld, stride, pos, stride_pos, batch, S, heads, base):
        _lib.check(self.lib.m3s_vit_rope(_p(t), ld, stride, _p(pos), stride_pos, batch, S, heads,
                                         float(base), self._s()), "vit_rope")

    def rope_table(self, pos, base):
        """pos int64 [S,2] → f32 [S,2,2,16] cos/sin table for the GEMM-epilogue RoPE."""
        tab = torch.empty((pos.shape[0], 2, 2, 16), dtype=F32, device=self.dev)
        _lib.check(self.lib.m3s_vit_rope_table(_p(pos), pos.shape[0], float(base), _p(tab),
                                               self._s()), "vit_rope_table")
        return tab

    def attn(self, q, ldq, sq_b, k, v, ldkv, skv_b, o, ldo, so_b, batch, heads, sq, sk,
             kv_xor=0):
        """kv_xor = 1: batch b reads k / v of batch b ^ 1."""
        ws = self.ws
        _lib.check(self.lib.m3s_vit_attention(_p(q), ldq, sq_b, _p(k), _p(v), ldkv, skv_b, None,
                                              None, 0, _p(o), ldo, so_b,
                                              int(o.element_size() == 1), batch, heads, sq, sk, 0.0,
                                              _p(ws), ws.numel(), kv_xor, self._s()),
                   "vit_attention")

    def copy_rows(self, src, dst, rows, row_bytes, src_row, dst_row, outer, inner, src_outer,
                  src_inner, src_base, dst_outer, dst_inner, dst_base):
        """m3s_copy_rows (byte strides): item (o, i) of outer x inner copies `rows` rows."""
        _lib.check(self.lib.m3s_copy_rows(_p(src), _p(dst), rows, row_bytes, src_row, dst_row,
                                          outer, inner, src_outer, src_inner, src_base,
                                          dst_outer, dst_inner, dst_base, self._s()), "copy_rows")

    def patchify(self, img, out, b, h, w):
        _lib.check(self.lib.m3s_vit_patchify(_p(img), _p(out), b, h, w, self._s()), "patchify")

    def up2(self, x, out, b, h, w, c, oh=None, ow=None, add=None, inv_scale=1.0):
        """out uint8 / float8_e4m3fn: e4m3 of the upsample times inv_scale."""
        if out.element_size() == 1:
            _lib.check(self.lib.m3s_vit_upsample2x_e4m3(
                _p(x), _p(out), _p(add), b, h, w, c, oh or 2 * h, ow or 2 * w, float(inv_scale),
                self._s()), "upsample2x_e4m3")
            return
        _lib.check(self.lib.m3s_vit_upsample2x(_p(x), _p(out), _p(add), b, h, w, c,
                                               oh or 2 * h, ow or 2 * w, self._s()), "upsample2x")

    def dpt_out(self, t, w4, b4, pts, conf, pixels, conf_min, batch, st, so, pmod=0):
        _lib.check(self.lib.m3s_vit_dpt_out(_p(t), _p(w4), _p(b4), _p(pts), _p(conf), pixels,
                                            float(conf_min), batch, st, so, pmod, self._s()),
                   "dpt_out")

    def local_features(self, feats, desc, desc16, dconf, b, h, w):
        _lib.check(self.lib.m3s_vit_local_features(_p(feats), _p(desc), _p(desc16), _p(dconf), b,
                                                   h, w, self._s()), "local_features")


# ---------------------------------------------------------------------------------------
# weight packing
# ---------------------------------------------------------------------------------------
def _drain(gen):
    """Run a launch-issuing generator to its end; its return value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


def _conv_pack(w):
    """[Cout][Cin][k][k] → [Cout][k][k][Cin] flattened (implicit-GEMM K order ky, kx, ci)."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def _convt_pack(w):
    """ConvTranspose [Cin][Cout][s][s] → [(a, b, co)][ci]."""
    return w.permute(2, 3, 1, 0).reshape(-1, w.shape[0])


def quant_e4m3(w):
    """Per-output-row symmetric e4m3 quantisation of a [.., N, K] weight stack:
    w ≈ q * scale[.., N, None], |q| ≤ 448.  Returns (q uint8 [.., N, K], scale f32 [.., N])."""
    w = w.float()
    sc = (w.abs().amax(-1) / 448.0).clamp_min(1e-12)
    q = (w / sc[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    return q.contiguous(), sc.contiguous()


def ln_fold(w, b, g, beta, dev):
    """LayerNorm → Linear folded for the LN_FOLD epilogue (croco/blocks.py: norm then
    projection): LN(x) Wᵀ + b = rstd (x (W∘γ)ᵀ − mean c1) + c2 with W' = bf16(W∘γ) (one
    rounding from the f32 weight), c1 = Σ_k W'[n,k] (of the rounded W', so the mean term
    cancels what the MFMA accumulates) and c2 = b + W β.  w [.., N, K], b [.., N],
    g / beta [.., K] (f32).  Returns (W' bf16, c1 f32, c2 f32) on dev."""
    w = w.to(device=dev, dtype=torch.float64)
    wf = (w * g.to(device=dev, dtype=torch.float64).unsqueeze(-2)).to(BF16).contiguous()
    c1 = wf.double().sum(-1).float().contiguous()
    c2 = (b.to(device=dev, dtype=torch.float64) +
          (w @ beta.to(device=dev, dtype=torch.float64).unsqueeze(-1)).squeeze(-1))
    return wf, c1, c2.float().contiguous()


# the transformer GEMMs that run on the fp8 MFMA in fp8 mode; patch embed,
# decoder_embed and the DPT/local-feature heads stay bf16
ENC_FP8 = ("qkv_w", "proj_w", "fc1_w", "fc2_w")
DEC_FP8 = ("qkv_w", "proj_w", "q_w", "kv_w", "cproj_w", "fc1_w", "fc2_w")
# ... and the DPT heads' two full-resolution 3x3 convs (round 5): their inputs are the
# bilinear upsamples (path1 → head.0, head.0 → head.2), which emit e4m3 directly
HEAD_FP8 = ("head0", "head2")
# ... and, for the fp8 LayerNorm fold (round 6), the gamma-folded norm → projection weights
ENC_FP8_FOLD = ("qkv_wf", "fc1_wf")
DEC_FP8_FOLD = ("qkvkv_wf", "q_wf", "fc1_wf")
FP8_ACT_HEADROOM = 2.0   # calibrated amax maps to 448 / 2: test frames may run hotter


def _assign_params(old, new):
    """`new` written into the tensors of dict `old` when every key, shape and dtype match
    (the tensors a captured graph reads stay the same), else `new` itself."""
    if (old.keys() != new.keys() or
            any(old[k].shape != new[k].shape or old[k].dtype != new[k].dtype for k in new)):
        return new
    for k in new:
        old[k].copy_(new[k])
    return old


def _fp8_shifted_params(W, cal):
    """Calibrated fp8 parameter copies (PairModel.calibrate_fp8): cal[(site, layer)] = the
    per-channel mean of that e4m3 operand ([C] for the encoder, [Z, C] per decoder problem;
    Z = 4 from the pair calibration).  Returns (encoder dict of [L, ...] stacks, decoder
    list of per-layer dicts of [4, ...] stacks), f32."""
    f64 = torch.float64
    mv = lambda w, mu: torch.einsum("...nk,...k->...n", w.to(f64), mu)  # noqa: E731

    def deq(q8, b):
        q, sc = q8
        return q.view(torch.float8_e4m3fn).to(f64) * sc.to(f64)[..., None] - b.to(f64)

    L = W.arch.enc_depth
    P, P8 = W.enc, W.enc8
    st = lambda site: torch.stack([cal[(site, i)] for i in range(L)])  # noqa: E731
    m1, ma, m2, mh = st("enc.ln1"), st("enc.att"), st("enc.ln2"), st("enc.hid")
    E = m1.shape[-1]
    enc = {"ln1_b": P["ln1_b"].to(f64) - m1, "ln2_b": P["ln2_b"].to(f64) - m2}
    qkv_b = P["qkv_b"].to(f64) + mv(P["qkv_w"], m1)
    qkv_b[:, 2 * E:] -= ma
    enc["qkv_b"] = qkv_b
    enc["proj_b"] = P["proj_b"].to(f64) + mv(P["proj_w"], ma)
    enc["fc1_b"] = P["fc1_b"].to(f64) + mv(P["fc1_w"], m2)
    enc["fc2_b"] = P["fc2_b"].to(f64) - mv(deq(P8["fc2_w"], P["fc2_w"]), mh)
    enc = {k: v.float().contiguous() for k, v in enc.items()}
    dec = []
    for i, (P, P8) in enumerate(zip(W.dec, W.dec8)):
        m1, ma, my, m2, mc, m3, mh = (cal[(s, i)] for s in (
            "dec.ln1", "dec.att", "dec.lny", "dec.ln2", "dec.catt", "dec.ln3", "dec.hid"))
        D = m1.shape[-1]
        d = {"ln1_b": P["ln1_b"].to(f64) - m1, "lny_b": P["lny_b"].to(f64) - my,
             "ln2_b": P["ln2_b"].to(f64) - m2, "ln3_b": P["ln3_b"].to(f64) - m3}
        qkv_b = P["qkv_b"].to(f64) + mv(P["qkv_w"], m1)
        qkv_b[:, 2 * D:] -= ma
        d["qkv_b"] = qkv_b
        d["proj_b"] = P["proj_b"].to(f64) + mv(P["proj_w"], ma)
        kv_b = P["kv_b"].to(f64) + mv(P["kv_w"], my)
        kv_b[:, D:] -= mc
        d["kv_b"] = kv_b
        d["q_b"] = P["q_b"].to(f64) + mv(P["q_w"], m2)
        d["cproj_b"] = P["cproj_b"].to(f64) + mv(P["cproj_w"], mc)
        d["fc1_b"] = P["fc1_b"].to(f64) + mv(P["fc1_w"], m3)
        d["fc2_b"] = P["fc2_b"].to(f64) - mv(deq(P8["fc2_w"], P["fc2_w"]), mh)
        dec.append({k: v.float().contiguous() for k, v in d.items()})
    return enc, dec


def _fp8_fold_params(W, cal, raw):
    """Parameters of the fp8 LayerNorm fold (round 6; PairModel._f8fold) from the same
    calibration pass as _fp8_shifted_params.  raw[(site, layer)] = (mean, max, min) per
    channel of the raw residual stream x where a LayerNorm reads it ([C] encoder, [4, C] per
    decoder weight stack).  The producer of that x writes e4m3((x − s)·qs) with s = the
    channel mean and qs = 448 / (headroom · max |x − s|); the consumer (gamma-folded weight
    W' of ln_fold, e4m3 per row with scale sw) then accumulates Σ (x − s)·W'q, dequantises
    with col_scale = sw / qs and adds c3 = W' s, so that the epilogue's
    rstd (acc − mean c1) + c2 is LN(x)·W'ᵀ + c2 up to the e4m3 roundings (c1, c3 from the
    bf16 W': the weight rounding meets only the centred x − s, as in the LayerNorm path).
    c2 of the q/k/v projections carries the attention-output shifts of _fp8_shifted_params
    (the v columns minus that attention's calibrated output mean).  Returns (encoder dict of
    [L, ...] stacks, decoder list of per-layer dicts of [4, ...] stacks), f32."""
    f64 = torch.float64

    def qscale(mean, mx, mn):   # one scale per (layer | stack): the largest channel range
        amax = torch.maximum(mx - mean, mean - mn)
        return 448.0 / (FP8_ACT_HEADROOM * amax.amax(-1).clamp_min(1e-30))

    def consumer(q8, wf, s, qs):   # (col_scale, c3) of a gamma-folded e4m3 weight
        return (q8[1].to(f64) / qs[..., None],
                torch.einsum("...nk,...k->...n", wf.to(f64), s))

    L = W.arch.enc_depth
    P, P8 = W.enc, W.enc8
    stk = lambda site, j: torch.stack([raw[(site, i)][j] for i in range(L)])  # noqa: E731
    s1, s2 = stk("enc.x1", 0), stk("enc.x2", 0)
    qs1 = qscale(s1, stk("enc.x1", 1), stk("enc.x1", 2))
    qs2 = qscale(s2, stk("enc.x2", 1), stk("enc.x2", 2))
    E = s1.shape[-1]
    ma = torch.stack([cal[("enc.att", i)] for i in range(L)])
    qkv_cs, qkv_c3 = consumer(P8["qkv_wf"], P["qkv_wf"], s1, qs1)
    fc1_cs, fc1_c3 = consumer(P8["fc1_wf"], P["fc1_wf"], s2, qs2)
    qkv_c2 = P["qkv_c2"].to(f64).clone()
    qkv_c2[:, 2 * E:] -= ma
    enc = dict(s1=s1, qs1=qs1, s2=s2, qs2=qs2, qkv_cs=qkv_cs, qkv_c3=qkv_c3, qkv_c2=qkv_c2,
               fc1_cs=fc1_cs, fc1_c3=fc1_c3, fc1_c2=P["fc1_c2"])
    enc = {k: v.float().contiguous() for k, v in enc.items()}
    dec = []
    sw = [1, 0, 3, 2]
    for i, (P, P8) in enumerate(zip(W.dec, W.dec8)):
        d = {}
        for t in ("1", "2", "3"):
            mean, mx, mn = raw[("dec.x" + t, i)]
            d["s" + t], d["qs" + t] = mean, qscale(mean, mx, mn)
        D = d["s1"].shape[-1]
        d["qkvkv_cs"], d["qkvkv_c3"] = consumer(P8["qkvkv_wf"], P["qkvkv_wf"], d["s1"], d["qs1"])
        d["q_cs"], d["q_c3"] = consumer(P8["q_wf"], P["q_wf"], d["s2"], d["qs2"])
        d["fc1_cs"], d["fc1_c3"] = consumer(P8["fc1_wf"], P["fc1_wf"], d["s3"], d["qs3"])
        # fused columns [q | k | k' | v | v']: v = this problem's self-attention, v' = the
        # cross-attention values of problem z ^ 1 (PackedWeights "qkvkv")
        c2 = P["qkvkv_c2"].to(f64).clone()
        c2[:, 3 * D:4 * D] -= cal[("dec.att", i)]
        c2[:, 4 * D:] -= cal[("dec.catt", i)][sw]
        d["qkvkv_c2"] = c2
        d["q_c2"], d["fc1_c2"] = P["q_c2"], P["fc1_c2"]
        dec.append({k: v.float().contiguous() for k, v in d.items()})
    return enc, dec


class PackedWeights:
    """Device weights.  Encoder from MonST3R; decoders and heads stacked over
    z = model*2 + side (model 0 = MonST3R, 1 = MASt3R; side 0 = dec_blocks/head1,
    side 1 = dec_blocks2/head2)."""

    def __init__(self, sd_monst3r, arch_monst3r, sd_mast3r, arch_mast3r, device):
        am, aM = arch_monst3r, arch_mast3r
        assert (am.enc_dim, am.dec_dim, am.enc_depth, am.dec_depth) == \
               (aM.enc_dim, aM.dec_dim, aM.enc_depth, aM.dec_depth)
        self.arch, self.arch_mast3r = am, aM
        dev = device
        bf = lambda t: t.to(device=dev, dtype=BF16).contiguous()  # noqa: E731
        f32 = lambda t: t.to(device=dev, dtype=F32).contiguous()  # noqa: E731
        sdm = sd_monst3r
        E, L = am.enc_dim, am.enc_depth
        # ---- encoder (MonST3R weights only: monst3r_utils.py:262-269) ----
        self.patch_w = bf(sdm["patch_embed.proj.weight"].reshape(E, -1))
        self.patch_b = f32(sdm["patch_embed.proj.bias"])
        st = lambda key: torch.stack([sdm[f"enc_blocks.{i}.{key}"] for i in range(L)])  # noqa
        self.enc = dict(
            ln1_g=f32(st("norm1.weight")), ln1_b=f32(st("norm1.bias")),
            qkv_w=bf(st("attn.qkv.weight")), qkv_b=f32(st("attn.qkv.bias")),
            proj_w=bf(st("attn.proj.weight")), proj_b=f32(st("attn.proj.bias")),
            ln2_g=f32(st("norm2.weight")), ln2_b=f32(st("norm2.bias")),
            fc1_w=bf(st("mlp.fc1.weight")), fc1_b=f32(st("mlp.fc1.bias")),
            fc2_w=bf(st("mlp.fc2.weight")), fc2_b=f32(st("mlp.fc2.bias")))
        # LayerNorm-folded copies of the norm → projection pairs (ln_fold): qkv ← norm1,
        # fc1 ← norm2 → keys <name>_wf / _c1 / _c2
        for name, lin, nrm in (("qkv", "attn.qkv", "norm1"), ("fc1", "mlp.fc1", "norm2")):
            wf, c1, c2 = ln_fold(st(lin + ".weight"), st(lin + ".bias"), st(nrm + ".weight"),
                                 st(nrm + ".bias"), dev)
            self.enc.update({name + "_wf": wf, name + "_c1": c1, name + "_c2": c2})
        self.enc_norm_g = f32(sdm["enc_norm.weight"])
        self.enc_norm_b = f32(sdm["enc_norm.bias"])
        # ---- decoders, z = model*2 + side ----
        sds = [sd_monst3r, sd_monst3r, sd_mast3r, sd_mast3r]
        blk = ["dec_blocks", "dec_blocks2", "dec_blocks", "dec_blocks2"]

        def dz(key, layer=None):
            ts = []
            for z in range(4):
                name = key if layer is None else f"{blk[z]}.{layer}.{key}"
                ts.append(sds[z][name])
            return torch.stack(ts)

        self.dec_embed_w = bf(dz("decoder_embed.weight"))
        self.dec_embed_b = f32(dz("decoder_embed.bias"))
        self.dec = []
        for i in range(am.dec_depth):
            kv_w = torch.cat([dz("cross_attn.projk.weight", i), dz("cross_attn.projv.weight", i)], 1)
            kv_b = torch.cat([dz("cross_attn.projk.bias", i), dz("cross_attn.projv.bias", i)], 1)
            self.dec.append(dict(
                ln1_g=f32(dz("norm1.weight", i)), ln1_b=f32(dz("norm1.bias", i)),
                qkv_w=bf(dz("attn.qkv.weight", i)), qkv_b=f32(dz("attn.qkv.bias", i)),
                proj_w=bf(dz("attn.proj.weight", i)), proj_b=f32(dz("attn.proj.bias", i)),
                ln2_g=f32(dz("norm2.weight", i)), ln2_b=f32(dz("norm2.bias", i)),
                lny_g=f32(dz("norm_y.weight", i)), lny_b=f32(dz("norm_y.bias", i)),
                q_w=bf(dz("cross_attn.projq.weight", i)), q_b=f32(dz("cross_attn.projq.bias", i)),
                kv_w=bf(kv_w), kv_b=f32(kv_b),
                cproj_w=bf(dz("cross_attn.proj.weight", i)),
                cproj_b=f32(dz("cross_attn.proj.bias", i)),
                ln3_g=f32(dz("norm3.weight", i)), ln3_b=f32(dz("norm3.bias", i)),
                fc1_w=bf(dz("mlp.fc1.weight", i)), fc1_b=f32(dz("mlp.fc1.bias", i)),
                fc2_w=bf(dz("mlp.fc2.weight", i)), fc2_b=f32(dz("mlp.fc2.bias", i))))
            # LayerNorm-folded copies: qkv ← norm1, kv ← norm_y (of the other side's x),
            # q ← norm2, fc1 ← norm3
            P = self.dec[-1]
            for name, w, b, nrm in (
                    ("qkv", dz("attn.qkv.weight", i), dz("attn.qkv.bias", i), "norm1"),
                    ("kv", kv_w, kv_b, "norm_y"),
                    ("q", dz("cross_attn.projq.weight", i), dz("cross_attn.projq.bias", i), "norm2"),
                    ("fc1", dz("mlp.fc1.weight", i), dz("mlp.fc1.bias", i), "norm3")):
                wf, c1, c2 = ln_fold(w, b, dz(nrm + ".weight", i), dz(nrm + ".bias", i), dev)
                P.update({name + "_wf": wf, name + "_c1": c1, name + "_c2": c2})
            # self-attention qkv of problem z and the cross-attention k/v that problem z ^ 1
            # takes from z's tokens (norm_y params / weights of z ^ 1) read the same A rows:
            # one GEMM, output columns [q | k | k' | v | v'] (RoPE on the first 3 blocks)
            D = am.dec_dim
            sw = [1, 0, 3, 2]

            def fuse(a, b):
                b = b[sw]
                return torch.cat([a[:, :2 * D], b[:, :D], a[:, 2 * D:], b[:, D:]], 1).contiguous()
            for suf in ("_wf", "_c1", "_c2"):
                P["qkvkv" + suf] = fuse(P.pop("qkv" + suf), P.pop("kv" + suf))
        self.dec_norm_g = f32(dz("dec_norm.weight"))
        self.dec_norm_b = f32(dz("dec_norm.bias"))
        # ---- DPT heads, z = model*2 + side ----
        hd = ["downstream_head1", "downstream_head2", "downstream_head1", "downstream_head2"]

        def hz(key, pack=None):
            ts = []
            for z in range(4):
                t = sds[z][f"{hd[z]}.dpt.{key}"]
                ts.append(pack(t) if pack else t)
            return torch.stack(ts)

        ap = "act_postprocess."
        self.h = dict(
            ap0_w=bf(hz(ap + "0.0.weight", _conv_pack)), ap0_b=f32(hz(ap + "0.0.bias")),
            ap0t_w=bf(hz(ap + "0.1.weight", _convt_pack)), ap0t_b=f32(hz(ap + "0.1.bias")),
            ap1_w=bf(hz(ap + "1.0.weight", _conv_pack)), ap1_b=f32(hz(ap + "1.0.bias")),
            ap1t_w=bf(hz(ap + "1.1.weight", _convt_pack)), ap1t_b=f32(hz(ap + "1.1.bias")),
            ap2_w=bf(hz(ap + "2.0.weight", _conv_pack)), ap2_b=f32(hz(ap + "2.0.bias")),
            ap3_w=bf(hz(ap + "3.0.weight", _conv_pack)), ap3_b=f32(hz(ap + "3.0.bias")),
            ap3c_w=bf(hz(ap + "3.1.weight", _conv_pack)), ap3c_b=f32(hz(ap + "3.1.bias")),
            head0_w=bf(hz("head.0.weight", _conv_pack)), head0_b=f32(hz("head.0.bias")),
            head2_w=bf(hz("head.2.weight", _conv_pack)), head2_b=f32(hz("head.2.bias")),
            head4_w=f32(hz("head.4.weight", lambda t: t.reshape(t.shape[0], -1))),
            head4_b=f32(hz("head.4.bias")))
        for k in range(4):
            self.h[f"rn{k}_w"] = bf(hz(f"scratch.layer{k + 1}_rn.weight", _conv_pack))
        for k in range(1, 5):
            q = f"scratch.refinenet{k}."
            self.h[f"r{k}_out_w"] = bf(hz(q + "out_conv.weight", _conv_pack))
            self.h[f"r{k}_out_b"] = f32(hz(q + "out_conv.bias"))
            for u in (1, 2):
                for c in (1, 2):
                    key = f"resConfUnit{u}.conv{c}"
                    self.h[f"r{k}_u{u}c{c}_w"] = bf(hz(q + key + ".weight", _conv_pack))
                    self.h[f"r{k}_u{u}c{c}_b"] = f32(hz(q + key + ".bias"))
        # ---- MASt3R local features (model 1 only: z = 2, 3) ----
        lf = ["downstream_head1", "downstream_head2"]
        self.lf_fc1_w = bf(torch.stack([sd_mast3r[f"{h}.head_local_features.fc1.weight"] for h in lf]))
        self.lf_fc1_b = f32(torch.stack([sd_mast3r[f"{h}.head_local_features.fc1.bias"] for h in lf]))
        self.lf_fc2_w = bf(torch.stack([sd_mast3r[f"{h}.head_local_features.fc2.weight"] for h in lf]))
        self.lf_fc2_b = f32(torch.stack([sd_mast3r[f"{h}.head_local_features.fc2.bias"] for h in lf]))
        self.enc8 = self.dec8 = None
        self.fp8_shift_enc, self.fp8_shift_dec = {}, [{} for _ in self.dec]
        self.fp8_fold_enc, self.fp8_fold_dec = {}, [{} for _ in self.dec]
        self.fp8_calibrated = False
        self.h8, self.h8_cs, self.h8_inv = None, {}, {}

    def enable_fp8(self):
        """e4m3 copies (+ per-row scales) of the encoder / decoder transformer weights,
        quantised from the bf16 packs (the bf16 packs stay for the bf16 path)."""
        if self.enc8 is None:
            self.enc8 = {k: quant_e4m3(self.enc[k]) for k in ENC_FP8}
            self.dec8 = [{k: quant_e4m3(P[k]) for k in DEC_FP8} for P in self.dec]
            # the DPT heads' full-resolution convs (head.0, head.2: Cin 256 / 128, packed
            # [Cout][ky][kx][Cin] rows), per-Cout scales; their e4m3 inputs come from the
            # upsample with a calibrated per-tensor scale (h8_cs = row scale x act scale)
            self.h8 = {k: quant_e4m3(self.h[k + "_w"]) for k in HEAD_FP8}
            # the gamma-folded projections of the LayerNorm fold (ln_fold), e4m3 per row
            self.enc8.update({k: quant_e4m3(self.enc[k]) for k in ENC_FP8_FOLD})
            for P, P8 in zip(self.dec, self.dec8):
                P8.update({k: quant_e4m3(P[k]) for k in DEC_FP8_FOLD})


# ---------------------------------------------------------------------------------------
# model runner
# ---------------------------------------------------------------------------------------
def _exp_hot_weights(part):
    """DIAGNOSTIC ONLY (wrong outputs; tools / sweeps): M3S_EXP_HOT_WEIGHTS = enc | dec |
    both makes every block of that stack read block 0's weights, so they stay cache-
    resident across the step — how much of the step waits on streaming the weights."""
    v = os.environ.get("M3S_EXP_HOT_WEIGHTS", "")
    return v == part or v == "both"


def _tile_knob(env, names, default):
    """GEMM tile hints {projection: (TileCfg, split-K)} from an experiment knob: "cfg:splits"
    for every projection, "name=cfg:splits,..." for some (the others: per-shape table),
    "table" for none; unset → default."""
    knob = os.environ.get(env)
    if not knob:
        return default
    tiles = {}
    if knob != "table":
        for part in knob.split(","):
            name, _, val = part.rpartition("=")
            cfg, _, sp = val.partition(":")
            for n in ([name] if name else names):
                tiles[n] = (int(cfg), int(sp or 1))
    return tiles


class PairModel:
    """Frame/keyframe pair inference.  Buffers are allocated once per image size."""

    def __init__(self, packed: PackedWeights, device):
        self.w = packed
        self.a = packed.arch
        self.dev = device
        self.ops = Ops(device)
        self._bufs = {}
        # Independent chains run on side streams (captured into the same HIP graph): the
        # decoder's norm_y + k/v projection overlap the self-attention half of the layer,
        # the MASt3R local-feature MLP overlaps the DPT heads, the DPT's four
        # act_postprocess branches run concurrently — when `serial` is False.  Measured on
        # the tracking step (tools/gpu_cmd_r1y.sh): the side-stream kernels take CUs from
        # the critical path and the graph gains dependency edges, 118.5 vs 124.9 frames/s
        # serial, so one stream is the default.
        self.side = [torch.cuda.Stream(device), torch.cuda.Stream(device)]
        self.serial = True
        self.fp8 = False
        self.fp8_convs = os.environ.get("M3S_FP8_CONVS", "0") == "1"
        # bf16 path: the blocks' LayerNorms folded into the following projections (ln_fold;
        # LN_STATS / LN_FOLD epilogues) instead of separate LayerNorm launches
        self.lnfold = os.environ.get("M3S_LNFOLD", "1") != "0"
        # fp8 path: the same fold on e4m3 operands (shifted e4m3 copy of x from the residual
        # GEMMs, calibrated shifts / scales; _fp8_fold_params) — M3S_FP8_FOLD=0: separate
        # e4m3 LayerNorm launches as in round 5
        self.fp8_fold = os.environ.get("M3S_FP8_FOLD", "1") != "0"
        # tile configurations (TileCfg, split-K) of the prefetched encoder's projections,
        # measured in the pipelined C3 step (encode(concurrent=True)); {} = per-shape table
        # (T128W8 residual GEMMs: 212.8 → 224.5 frames/s; with the split decoder, T256W8
        # qkv / fc1: 214.9 → 221.3, profiles/r02_enc_tile_sweep.txt)
        # round 3, two-frame encoder (M = 1536) in the step: fc1 on the 256² tile,
        # proj / fc2 on 256x128: 238.2 → 242.8 frames/s (profiles/r03_sched_sweep_b.txt)
        self.enc_tiles_concurrent = {"qkv": (13, 1), "proj": (13, 1), "fc1": (14, 1),
                                     "fc2": (13, 1)}
        self.dec_tiles = {}   # decoder projections' tile hints (M3S_DEC_TILE; {} = table)
        # ... of the per-model split decoder (two batch-2 chains beside the prefetched
        # encoder), measured in the pipelined step: 226.9 → 232.7 frames/s
        self.dec_tiles_split = {"qkv": (13, 1), "fc2": (12, 1)}
        self.side_tiles = {}  # split-heads side chain (M3S_SIDE_TILE: lf / dpt; {} = table)
        # the pair decoder split by model onto two streams (decode_multi; M3S_DEC_SPLIT=0
        # restores the single batch-4 chain): 214.0 → 218.3 frames/s (2 × A/B)
        self.dec_split = os.environ.get("M3S_DEC_SPLIT", "1") == "1"
        # split heads: the local-feature MLP runs on the side chain ahead of the MASt3R heads
        self.lf_side = os.environ.get("M3S_LF_SIDE", "1") != "0"
        self._tag = None      # buffer-key prefix of the head set being issued (split heads)
        self._wbase = 0       # first head-weight stack of that set
        self._wm = 4
        self._ev_heads = None
        self.sym_chunk = 7    # most pairs per symmetric() launch set (8 problems each)

    def set_fp8(self, on=True, calibrate=True, convs=None):
        """fp8 mode: the encoder / decoder transformer GEMMs take OCP e4m3
        operands on the scaled MFMA — LayerNorm, attention and the fc1 GELU epilogue emit
        e4m3 activations (unscaled, saturated to ±448), weights are per-row scaled, the
        residual stream stays f32 and q/k/v stay bf16 (attention runs in bf16).
        calibrate: on first use, per-channel activation shifts and bias correction from two
        synthetic calibration frames (calibrate_fp8).
        convs: also run the DPT heads' two full-resolution convs (head.0, head.2) on the
        fp8 MFMA (e4m3 upsample outputs with a calibrated per-tensor scale).  Off by default:
        measured on the C5 frame 10.10 → 9.74 ms for pointmap error 2.85 → 5.41 % (pair X
        median, 512x512).  None keeps the current setting (M3S_FP8_CONVS=1
        turns it on for the bench / sweeps)."""
        if on:
            self.w.enable_fp8()
        if convs is not None:
            self.fp8_convs = bool(convs)
        self.fp8 = bool(on)
        if on and calibrate and not self.w.fp8_calibrated:
            self.calibrate_fp8()

    def calibrate_fp8(self, hw=(512, 512), frames=2, seed=100, images=None):
        """Static per-channel calibration of the fp8 path (round 5; tools/fp8_error_budget.py,
        tools/fp8_mono_diag.py).  The e4m3 errors are not noise: a channel whose activation
        sits near a constant over all tokens rounds the same way in every token, and a
        quantised weight row meets the same per-channel input mean in every token, so both
        errors come out as a per-channel offset of the features (88 % of the fp8 encoder's
        feature error energy at 512x512).  Measured means mu (over the tokens of `frames`
        uniform-noise frames, seeds `seed`.., never the test frames) are folded into
        parameters — no kernel changes:
          LayerNorm -> GEMM   beta' = beta - mu, b' = b + W mu (the e4m3 operand carries
                              x - mu; W exact)
          attention -> proj   the v bias - mu (softmax rows sum to 1, so the output shifts
                              by -mu), b' = b + W mu
          GELU -> fc2         b' = b - (Wq - W) mu (bias correction of the quantised rows)
        In the fake-quant restatement: X median 5.5 % -> 1.9 %, feature cosine 0.99597 ->
        0.99936 (mono 512x512).  images: calibration frames [n >= 2, 3, H, W] in [-1, 1]
        (frames of the target domain with real checkpoints) instead of the noise frames."""
        W, dev = self.w, self.dev
        was, was_convs = self.fp8, self.fp8_convs
        old = (W.fp8_shift_enc, W.fp8_shift_dec)
        bufs_before = set(self._bufs)
        self.fp8 = True
        # the heads run their bf16 convs while calibrating: the amax of an e4m3 upsample
        # output would be its largest byte code, not its largest activation
        self.fp8_convs = False
        W.fp8_shift_enc, W.fp8_shift_dec = {}, [{} for _ in W.dec]   # plain biases first
        self._cal = {}
        try:
            if images is not None:
                img = images.to(device=dev, dtype=torch.float32)
                if img.dim() != 4 or img.shape[0] < 2:
                    raise ValueError("calibrate_fp8: images must be [n >= 2, 3, H, W]")
                frames, hw = img.shape[0], tuple(img.shape[-2:])
            else:
                gen = torch.Generator(device=dev).manual_seed(seed)
                img = torch.rand(frames, 3, hw[0], hw[1], device=dev, generator=gen) * 2 - 1
            feat, _ = self.encode(img)
            gh, gw = hw[0] // self.a.patch, hw[1] // self.a.patch
            f = feat.reshape(frames, gh * gw, self.a.enc_dim)
            # pairs (frame k, frame k+1): both models, both sides
            hooks = self.decode_multi(f.contiguous(), f.roll(1, 0).contiguous(), gh, gw)
            # the heads (bf16 convs) for the upsample outputs' amax
            self.heads(hooks, gh, gw, hw[0], hw[1])
            torch.cuda.synchronize(dev)
            amax = {k: float(v) for k, v in self._cal.items() if k[0] == "amax"}
            raw = {k[1:]: (v[0] / v[1], v[2], v[3]) for k, v in self._cal.items()
                   if k[0] == "raw"}
            cal = {k: v[0] / v[1] for k, v in self._cal.items() if k[0] not in ("amax", "raw")}
            enc, dec = _fp8_shifted_params(W, cal)
            fenc, fdec = _fp8_fold_params(W, cal, raw)
        except BaseException:
            # a failed calibration leaves the previous parameters in force
            W.fp8_shift_enc, W.fp8_shift_dec = old
            raise
        finally:
            self._cal = None
            self.fp8, self.fp8_convs = was, was_convs
            # calibration scratch (frame-count / size-specific buffers) is not kept: only
            # the buffers this call created are dropped, so graphs captured before it stay
            # valid (> 1 GB held for good after set_fp8)
            for k in set(self._bufs) - bufs_before:
                del self._bufs[k]
        # new values written into the tensors already in use where the layout matches, so
        # a graph captured in fp8 mode before a re-calibration replays the new parameters
        # (a changed layout allocates afresh: re-capture after a re-calibration then)
        W.fp8_shift_enc = _assign_params(old[0], enc)
        W.fp8_shift_dec = [_assign_params(o, n) for o, n in zip(old[1], dec)] \
            if len(old[1]) == len(dec) else dec
        W.fp8_fold_enc = _assign_params(W.fp8_fold_enc, fenc)
        W.fp8_fold_dec = [_assign_params(o, n) for o, n in zip(W.fp8_fold_dec, fdec)] \
            if len(W.fp8_fold_dec) == len(fdec) else fdec
        for k in HEAD_FP8:
            sc = max(amax[("amax", k)], 1e-30) * FP8_ACT_HEADROOM / 448.0
            W.h8_inv[k] = 1.0 / sc
            cs = (W.h8[k][1] * sc).contiguous()
            prev = W.h8_cs.get(k)
            if prev is not None and prev.shape == cs.shape and prev.dtype == cs.dtype:
                prev.copy_(cs)
            else:
                W.h8_cs[k] = cs
        W.fp8_calibrated = True

    def _calib(self, site, i, t, z=None):
        """Calibration hook: accumulate the per-channel mean of e4m3 operand t (rows ×
        channels, or [Z, S, C] per problem z when z is given)."""
        if getattr(self, "_cal", None) is None:
            return
        v = t.view(torch.float8_e4m3fn).double()
        C = v.shape[-1]
        if z is None:
            m = v.reshape(-1, C).mean(0)
        else:   # problems z = (g·models + model)·2 + side read weight stack z % wm
            m = v.reshape(z, -1, C).mean(1).reshape(-1, self._wm, C).mean(0)
        key = (site, i)
        acc, n = self._cal.get(key, (0.0, 0))
        self._cal[key] = (acc + m, n + 1)

    def _calib_raw(self, site, i, x, z=None):
        """Calibration hook of the fp8 LayerNorm fold: per-channel mean, max and min of the
        raw residual stream x (f32, rows × channels or [Z, S, C] per problem z) where a
        LayerNorm reads it (_fp8_fold_params)."""
        if getattr(self, "_cal", None) is None:
            return
        C = x.shape[-1]
        if z is None:
            v = x.reshape(-1, C)
            m, mx, mn = v.double().mean(0), v.amax(0).double(), v.amin(0).double()
        else:
            v = x.reshape(z, -1, C)
            m = v.double().mean(1).reshape(-1, self._wm, C).mean(0)
            mx = v.amax(1).double().reshape(-1, self._wm, C).amax(0)
            mn = v.amin(1).double().reshape(-1, self._wm, C).amin(0)
        key = ("raw", site, i)
        if key in self._cal:
            acc, n, pmx, pmn = self._cal[key]
            m, mx, mn = acc + m, torch.maximum(pmx, mx), torch.minimum(pmn, mn)
        else:
            n = 0
        self._cal[key] = (m, n + 1, mx, mn)

    def _f8fold(self):
        """fp8 mode with the LayerNorms folded into the e4m3 projections (round 6): calibrated,
        not calibrating, the fold on (M3S_LNFOLD) and M3S_FP8_FOLD != 0."""
        return (self.fp8 and self.fp8_fold and self.lnfold and self.w.fp8_calibrated and
                bool(self.w.fp8_fold_enc) and getattr(self, "_cal", None) is None)

    def _calib_amax(self, name, t):
        if getattr(self, "_cal", None) is not None:
            if t.dtype == torch.uint8:   # e4m3 bytes: not an activation range
                raise RuntimeError(f"calibrate_fp8: {name} is an e4m3 tensor")
            prev = self._cal.get(("amax", name), 0.0)
            self._cal[("amax", name)] = max(prev, float(t.float().abs().max()))

    def _fp8_convs(self):
        """The DPT head convs on the fp8 MFMA: fp8 mode with convs on (set_fp8), calibrated."""
        F = self.a.feature_dim
        # (the fp8 implicit conv takes Cin % 128 == 0: head.0 reads F, head.2 F / 2 channels)
        return (self.fp8 and self.fp8_convs and self.w.fp8_calibrated and
                self.w.h8 is not None and F % 256 == 0)

    def _conv3_f8(self, x, key, out, b, hin, win, cin, cout, bias_key=None, flags=0, dpt=None):
        """3x3 stride-1 conv on the fp8 MFMA: x e4m3 NHWC (scaled by h8_inv[key]), weights
        e4m3 per-Cout rows; the column scales undo both."""
        o, H, W = self.ops, self._hw, self.w
        q, cs = W.h8[key][0], W.h8_cs[key]
        if self._wbase:
            q, cs = q[self._wbase:], cs[self._wbase:]
        o.gemm(x, q, out, hin * win, cout, 9 * cin, b, sA=hin * win * cin, sB=cout * 9 * cin,
               sC=hin * win * cout, bias=H(bias_key) if bias_key else None, sBias=cout,
               flags=flags, conv=(hin, win, cin, hin, win, 1), wmod=self._wm, dpt=dpt,
               fp8=(cs, cout))

    def _pb(self, P, key, i=None, layer=None):
        """Bias / LayerNorm beta `key`: the fp8 path's calibrated copy when fp8 is on."""
        if self.fp8:
            Q = self.w.fp8_shift_enc if layer is None else self.w.fp8_shift_dec[layer]
            if key in Q:
                return Q[key] if i is None else Q[key][i]
        return P[key] if i is None else P[key][i]

    def _wt(self, P, P8, key, i=None, n=None):
        """(B operand, extra gemm kwargs) for weight `key` (layer i of a stacked pack, or
        the z-stack with per-problem scales of stride n)."""
        if not self.fp8 or key not in P8:
            return (P[key] if i is None else P[key][i]), {}
        q, sc = P8[key]
        if i is None:
            return q, dict(fp8=(sc, n))
        return q[i], dict(fp8=(sc[i], 0))

    # ---- streams ----
    def _on(self, k):
        """Context: launch on side stream k (after everything queued so far on the current
        stream), or on the current stream when serial."""
        if self.serial:
            return _Nullctx()
        main = torch.cuda.current_stream(self.dev)
        self.side[k].wait_stream(main)
        return torch.cuda.stream(self.side[k])

    def _event(self):
        if self.serial:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        return ev

    def _wait(self, ev):
        if ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(ev)

    # ---- buffers ----
    def _buf(self, key, shape, dtype):
        """Persistent scratch per (name, shape, dtype): a buffer is never freed or
        reallocated, so HIP graphs captured over it stay valid when other batch sizes run."""
        k = (self._tag, key, tuple(shape), dtype)
        t = self._bufs.get(k)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=self.dev)
            self._bufs[k] = t
        return t

    def positions(self, b, gh, gw):
        key = ("pos", b, gh, gw)
        t = self._bufs.get(key)
        if t is None:
            y = torch.arange(gh, device=self.dev)
            x = torch.arange(gw, device=self.dev)
            t = torch.cartesian_prod(y, x).view(1, gh * gw, 2).expand(b, -1, 2).contiguous()
            self._bufs[key] = t
        return t

    def rope_tab(self, gh, gw):
        key = ("rope", gh, gw)
        t = self._bufs.get(key)
        if t is None:
            t = self.ops.rope_table(self.positions(1, gh, gw)[0].contiguous(), self.a.rope_base)
            self._bufs[key] = t
        return t

    # ---- encoder: PatchEmbed + 24 blocks + enc_norm (batch of B images as M = B*S) ----
    def encode(self, img, out=None, concurrent=False):
        """img f32 [B,3,H,W] → feat bf16 [B,S,E], pos int64 [B,S,2].
        concurrent: this encoder shares the chip with the tracking chain (the next frame's
        prefetch, frontend.FramePipeline): its GEMMs take the tile configurations of
        `enc_tiles_concurrent` (measured in the pipelined C3 step) instead of the
        per-shape table, which is tuned for launches that have the chip to themselves.
        M3S_ENC_TILE (experiment knob, tools/enc_tile_sweep.sh): "cfg:splits" for all four
        projections, or "qkv=cfg:splits,proj=...,fc1=...,fc2=..."; "table" = no hints."""
        tiles = _tile_knob("M3S_ENC_TILE", ("qkv", "proj", "fc1", "fc2"),
                           self.enc_tiles_concurrent if concurrent else {})
        return self._encode(img.shape, img, out, tiles)

    def encode_part(self, shape, part, parts, img=None, out=None):
        """Part `part` of `parts` of a prefetched encode (concurrent tile hints) of a batch of
        `shape` = [B,3,H,W] images: part 0 embeds `img` and runs the first depth/parts blocks,
        the last part runs the remaining blocks and writes enc_norm into `out` [B,S,E].  The
        residual stream stays in this model's persistent buffers between the parts, so the
        parts may be issued in different captured graphs (frontend.FramePipeline(group=2)
        spreads a two-frame encode over two tracking steps).  Launch for launch the same work
        as encode(img, out, concurrent=True)."""
        tiles = _tile_knob("M3S_ENC_TILE", ("qkv", "proj", "fc1", "fc2"),
                           self.enc_tiles_concurrent)
        d = self.a.enc_depth
        lo, hi = d * part // parts, d * (part + 1) // parts
        g = self._encode_gen(shape, img if part == 0 else None,
                             out if part == parts - 1 else None, tiles, (lo, hi),
                             begin=part == 0, end=part == parts - 1)
        return _drain(g)

    def _encode(self, *args, **kw):
        return _drain(self._encode_gen(*args, **kw))

    def _encode_gen(self, shape, img=None, out=None, tiles=None, layers=None, begin=True,
                    end=True):
        """(Generator: yields after issuing each block; returns (feat, pos).)"""
        o, a, W = self.ops, self.a, self.w
        B, _, H, Wd = shape
        gh, gw = H // a.patch, Wd // a.patch
        S, E = gh * gw, a.enc_dim
        M = B * S
        lo, hi = layers if layers is not None else (0, a.enc_depth)
        patches = self._buf("enc_patch", (M, 3 * a.patch * a.patch), BF16)
        x = self._buf("enc_x", (M, E), F32)
        f8f = self._f8fold() and E % 128 == 0
        fold = self.lnfold and (not self.fp8 or f8f) and E % 128 == 0
        if fold:
            # LayerNorm folded into the projections (ln_fold): every residual-stream
            # producer also writes x in bf16 (fp8: e4m3 of x − shift, _fp8_fold_params) +
            # row statistics; no LayerNorm launches
            xb = self._buf("enc_xq" if f8f else "enc_xb", (M, E), U8 if f8f else BF16)
            st = self._buf("enc_stats", (M, E // 128, 2), F32)
            FE = self.w.fp8_fold_enc

            def lns(t, i):   # ln_stats of the producer of layer i's norm<t> input
                if not f8f:
                    return (xb, st)
                if i >= a.enc_depth:   # the last block's output goes to enc_norm
                    return None
                return (xb, st, FE["s" + t][i], FE["qs" + t][i:i + 1])
        if begin:
            img = img.to(F32).contiguous()
            o.patchify(img, patches, B, H, Wd)
            o.gemm(patches, W.patch_w, x, M, E, 3 * a.patch * a.patch, bias=W.patch_b,
                   flags=_lib.EPI_OUT_F32, ln_stats=lns("1", 0) if fold else None)
        adt = U8 if self.fp8 else BF16   # GEMM A operands: e4m3 bytes in fp8 mode
        xn = self._buf("enc_xn", (M, E), adt)
        qkv = self._buf("enc_qkv", (M, 3 * E), BF16)
        att = self._buf("enc_att", (M, E), adt)
        hid = self._buf("enc_hid", (M, a.mlp_ratio * E), adt)
        pos = self.positions(B, gh, gw)
        rt = self.rope_tab(gh, gw)
        P, P8 = W.enc, W.enc8
        R32 = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32
        for i in (range(lo, hi) if f8f else ()):
            # the fp8 fold: e4m3 gamma-folded qkv / fc1 on the shifted e4m3 copy of x
            o.gemm(xb, P8["qkv_wf"][0][i], qkv, M, 3 * E, E, bias=FE["qkv_c2"][i],
                   rope=(rt, 2 * E, S), ln_fold=(st, P["qkv_c1"][i], 0, FE["qkv_c3"][i]),
                   fp8=(FE["qkv_cs"][i], 0), tile=tiles.get("qkv"))
            o.attn(qkv, 3 * E, S * 3 * E, qkv[:, E:], qkv[:, 2 * E:], 3 * E, S * 3 * E, att,
                   E, S * E, B, a.enc_heads, S, S)
            w, kw = self._wt(P, P8, "proj_w", i)
            o.gemm(att, w, x, M, E, E, bias=self._pb(P, "proj_b", i), R=x, flags=R32,
                   ln_stats=lns("2", i), tile=tiles.get("proj"), **kw)
            o.gemm(xb, P8["fc1_wf"][0][i], hid, M, a.mlp_ratio * E, E, bias=FE["fc1_c2"][i],
                   flags=_lib.EPI_GELU, out_fp8=True,
                   ln_fold=(st, P["fc1_c1"][i], 0, FE["fc1_c3"][i]), fp8=(FE["fc1_cs"][i], 0),
                   tile=tiles.get("fc1"))
            w, kw = self._wt(P, P8, "fc2_w", i)
            o.gemm(hid, w, x, M, E, a.mlp_ratio * E, bias=self._pb(P, "fc2_b", i), R=x,
                   flags=R32, ln_stats=lns("1", i + 1), tile=tiles.get("fc2"), **kw)
            yield i
        if fold and not f8f:
            hot = _exp_hot_weights("enc")
            R32S = dict(flags=R32, ln_stats=(xb, st))
            for i in range(lo, hi):
                j = 0 if hot else i
                o.gemm(xb, P["qkv_wf"][j], qkv, M, 3 * E, E, bias=P["qkv_c2"][j],
                       rope=(rt, 2 * E, S), ln_fold=(st, P["qkv_c1"][j], 0), tile=tiles.get("qkv"))
                o.attn(qkv, 3 * E, S * 3 * E, qkv[:, E:], qkv[:, 2 * E:], 3 * E, S * 3 * E, att,
                       E, S * E, B, a.enc_heads, S, S)
                o.gemm(att, P["proj_w"][j], x, M, E, E, bias=P["proj_b"][j], R=x,
                       tile=tiles.get("proj"), **R32S)
                o.gemm(xb, P["fc1_wf"][j], hid, M, a.mlp_ratio * E, E, bias=P["fc1_c2"][j],
                       flags=_lib.EPI_GELU, ln_fold=(st, P["fc1_c1"][j], 0), tile=tiles.get("fc1"))
                o.gemm(hid, P["fc2_w"][j], x, M, E, a.mlp_ratio * E, bias=P["fc2_b"][j], R=x,
                       tile=tiles.get("fc2"), **R32S)
                yield i
        pb = self._pb
        for i in (range(lo, hi) if not fold else ()):
            self._calib_raw("enc.x1", i, x)
            o.ln(x, P["ln1_g"][i], pb(P, "ln1_b", i), xn, M, E)
            self._calib("enc.ln1", i, xn)
            # qkv projection with RoPE2D on q and k fused into the epilogue
            w, kw = self._wt(P, P8, "qkv_w", i)
            o.gemm(xn, w, qkv, M, 3 * E, E, bias=pb(P, "qkv_b", i), rope=(rt, 2 * E, S), **kw)
            o.attn(qkv, 3 * E, S * 3 * E, qkv[:, E:], qkv[:, 2 * E:], 3 * E, S * 3 * E, att, E,
                   S * E, B, a.enc_heads, S, S)
            self._calib("enc.att", i, att)
            w, kw = self._wt(P, P8, "proj_w", i)
            o.gemm(att, w, x, M, E, E, bias=pb(P, "proj_b", i), R=x,
                   flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, **kw)
            self._calib_raw("enc.x2", i, x)
            o.ln(x, P["ln2_g"][i], pb(P, "ln2_b", i), xn, M, E)
            self._calib("enc.ln2", i, xn)
            w, kw = self._wt(P, P8, "fc1_w", i)
            o.gemm(xn, w, hid, M, a.mlp_ratio * E, E, bias=pb(P, "fc1_b", i),
                   flags=_lib.EPI_GELU, out_fp8=self.fp8, **kw)
            self._calib("enc.hid", i, hid)
            w, kw = self._wt(P, P8, "fc2_w", i)
            o.gemm(hid, w, x, M, E, a.mlp_ratio * E, bias=pb(P, "fc2_b", i), R=x,
                   flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, **kw)
            yield i
        if not end:
            return None, pos
        feat = out if out is not None else torch.empty((B, S, E), dtype=BF16, device=self.dev)
        o.ln(x, W.enc_norm_g, W.enc_norm_b, feat, M, E)
        return feat, pos

    # ---- decoders: both models x both sides, batch z = model*2 + side ----
    def decode(self, feat_i, feat_j, pos, gh, gw, on_hook=None):
        """feat_i/feat_j bf16 [S,E] (frame i = side 1, keyframe j = side 2).
        Returns hooks dict: h0 bf16 [4,S,E], h6/h9/h12 bf16 [4,S,D] (h12 = dec_norm)."""
        S, E = gh * gw, self.a.enc_dim
        return self.decode_multi(feat_i.reshape(1, S, E), feat_j.reshape(1, S, E), gh, gw,
                                 on_hook=on_hook)

    def decode_multi(self, feat1, feat2, gh, gw, models=2, on_hook=None):
        """G directed pairs at once: feat1/feat2 bf16 [G,S,E] are the first / second view of
        each pair (d3r/model.py:171-190 `_decoder(f1, pos1, f2, pos2)`), decoded by BOTH
        models (models=2) or by MonST3R alone (models=1, the dynamic-mask mono decode).
        Problems z = (g*models + model)*2 + side; every launch covers all of them and reads
        the weight stack of z % (2*models) (weight_mod).  Returns hooks [2*models*G,S,*].
        on_hook(name, hooks): called as each hook (h0, h6, h9, h12) has been enqueued."""
        o, a, W = self.ops, self.a, self.w
        S, E, D = gh * gw, a.enc_dim, a.dec_dim
        G = feat1.shape[0]
        wm = 2 * models
        self._wm = wm
        Z = wm * G
        h0 = self._buf("h0", (Z, S, E), BF16)
        # h0[(g·models + m)·2 + side] = (feat1 | feat2)[g] for every model m: one row copy
        # per side (in-tree kernel), feat_* [G,S,E] contiguous
        fb = S * E * 2
        for side, f in ((0, feat1), (1, feat2)):
            f = f.reshape(G, S, E)
            if not f.is_contiguous():
                raise RuntimeError("decode_multi: features must be contiguous [G,S,E]")
            o.copy_rows(f, h0, 1, fb, fb, fb, G, models, fb, 0, 0, 2 * models * fb, 2 * fb,
                        side * fb)
        x = self._buf("dec_x", (Z, S, D), F32)
        f8f = self._f8fold()
        fold = self.lnfold and (not self.fp8 or f8f) and self.serial and D % 128 == 0
        lns = None
        if fold:
            # fp8: the residual stream's shifted e4m3 copy (_fp8_fold_params) instead of bf16
            xb = self._buf("dec_xq" if f8f else "dec_xb", (Z, S, D), U8 if f8f else BF16)
            st = self._buf("dec_stats", (Z, S, D // 128, 2), F32)
            F0 = W.fp8_fold_dec[0]
            lns = (xb, st, F0["s1"], F0["qs1"]) if f8f else (xb, st)
        o.gemm(h0, W.dec_embed_w, x, S, D, E, Z, sA=S * E, sB=D * E, sC=S * D,
               bias=W.dec_embed_b, sBias=D, flags=_lib.EPI_OUT_F32, wmod=wm, ln_stats=lns)
        if on_hook is not None:
            on_hook("h0", {"h0": h0})
        if fold and self.dec_split and models == 2 and G == 1 and on_hook is None:
            # the two models' decoders (z 0-1 MonST3R, 2-3 MASt3R: independent chains) as two
            # batch-2 chains on two streams, so each fills the other's kernel tails / gaps
            main = torch.cuda.current_stream(self.dev)
            # (the side chain's stream is the heads' side stream too: the decoder joins the
            # capture stream before any head is issued, so the step captures three streams —
            # DESIGN §5 "Capture topology")
            side = self.side[0]
            side.wait_stream(main)
            g0 = self._decode_folded_gen(x, xb, st, h0, Z, S, E, D, gh, gw, wm, None, part=0)
            g1 = self._decode_folded_gen(x, xb, st, h0, Z, S, E, D, gh, gw, wm, None, part=1)
            hooks = _drain(g0)
            with torch.cuda.stream(side):
                _drain(g1)
            main.wait_stream(side)
            h12 = self._buf("h12", (Z, S, D), BF16)
            o.ln(x, W.dec_norm_g, W.dec_norm_b, h12, S, D, Z, S * D, S * D, D, pmod=wm)
            hooks["h12"] = h12
            return hooks
        if fold:
            return self._decode_folded(x, xb, st, h0, Z, S, E, D, gh, gw, wm, on_hook)
        if (self.dec_split and models == 2 and G == 1 and on_hook is None and
                getattr(self, "_cal", None) is None):
            # the fp8 (unfolded) decoder split by model as the folded one above: two batch-2
            # chains, model 1 on side stream 0 (C5's pair decode, round 5)
            main = torch.cuda.current_stream(self.dev)
            side = self.side[0]
            side.wait_stream(main)
            g0 = self._decode_plain_gen(x, h0, Z, S, D, gh, gw, wm, None, part=0)
            g1 = self._decode_plain_gen(x, h0, Z, S, D, gh, gw, wm, None, part=1)
            hooks = _drain(g0)
            with torch.cuda.stream(side):
                _drain(g1)
            main.wait_stream(side)
        else:
            hooks = _drain(self._decode_plain_gen(x, h0, Z, S, D, gh, gw, wm, on_hook))
        h12 = self._buf("h12", (Z, S, D), BF16)
        o.ln(x, W.dec_norm_g, W.dec_norm_b, h12, S, D, Z, S * D, S * D, D, pmod=wm)
        hooks["h12"] = h12
        if on_hook is not None:
            on_hook("h12", hooks)
        return hooks

    def _decode_plain_gen(self, x, h0, Z, S, D, gh, gw, wm, on_hook=None, part=None):
        """(Generator: yields after issuing each block; returns the hooks h0, h6, h9 — the
        caller adds h12.)  decode_multi's blocks with separate LayerNorm launches: the fp8
        path (e4m3 LayerNorm / attention / GELU outputs as the fp8 GEMMs' A operands, the
        calibrated shifts of calibrate_fp8) and the bf16 path when the fold is off.
        part: one model's two problems (z in [2·part, 2·part + 2)), buffers, weights and
        calibrated parameters sliced, weight_mod 2."""
        o, a, W = self.ops, self.a, self.w
        adt = U8 if self.fp8 else BF16
        xn = self._buf("dec_xn", (Z, S, D), adt)
        yn = self._buf("dec_yn", (Z, S, D), adt)
        qkv = self._buf("dec_qkv", (Z, S, 3 * D), BF16)
        kv = self._buf("dec_kv", (Z, S, 2 * D), BF16)
        q = self._buf("dec_q", (Z, S, D), BF16)
        att = self._buf("dec_att", (Z, S, D), adt)
        hid = self._buf("dec_hid", (Z, S, a.mlp_ratio * D), adt)
        hook_bufs = {k: self._buf(f"h{k}", (Z, S, D), BF16) for k in a.hooks[1:3]}
        hooks = {"h0": h0}
        sl = None
        if part is not None:
            sl = slice(2 * part, 2 * part + 2)
            xn, yn, qkv, kv, q, att, hid, x = (t[sl] for t in (xn, yn, qkv, kv, q, att, hid, x))
            Z, wm = 2, 2
        rt = self.rope_tab(gh, gw)
        R32 = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32
        Dm = a.mlp_ratio * D
        for i in range(a.dec_depth):
            P = W.dec[i]
            P8 = W.dec8[i] if self.fp8 else None
            Q = W.fp8_shift_dec[i] if self.fp8 else {}
            if sl is not None:
                P = {k: v[sl] for k, v in P.items()}
                P8 = {k: (v[0][sl], v[1][sl]) for k, v in P8.items()} if P8 else None
                Q = {k: v[sl] for k, v in Q.items()}

            def wt(key, n, P=P, P8=P8):
                return self._wt(P, P8, key, None, n)

            def pb(key, P=P, Q=Q):   # bias / LayerNorm beta: the calibrated copy in fp8 mode
                return Q[key] if key in Q else P[key]
            # norm1(x) and norm_y(other side's x) share the row statistics: one pass; then
            # y_'s k/v projection
            w, kw = wt("kv_w", 2 * D)
            self._calib_raw("dec.x1", i, x, Z)
            o.ln_dual(x, P["ln1_g"], pb("ln1_b"), xn, P["lny_g"], pb("lny_b"), yn, S, D, Z,
                      S * D, S * D, D, pmod=wm)
            self._calib("dec.lny", i, yn, Z)
            o.gemm(yn, w, kv, S, 2 * D, D, Z, sA=S * D, sB=2 * D * D,
                   sC=S * 2 * D, bias=pb("kv_b"), sBias=2 * D, rope=(rt, D, S), wmod=wm, **kw)
            self._calib("dec.ln1", i, xn, Z)
            # self-attention
            w, kw = wt("qkv_w", 3 * D)
            o.gemm(xn, w, qkv, S, 3 * D, D, Z, sA=S * D, sB=3 * D * D, sC=S * 3 * D,
                   bias=pb("qkv_b"), sBias=3 * D, rope=(rt, 2 * D, S), wmod=wm, **kw)
            o.attn(qkv, 3 * D, S * 3 * D, qkv[:, :, D:], qkv[:, :, 2 * D:], 3 * D, S * 3 * D, att,
                   D, S * D, Z, a.dec_heads, S, S)
            self._calib("dec.att", i, att, Z)
            w, kw = wt("proj_w", D)
            o.gemm(att, w, x, S, D, D, Z, sA=S * D, sB=D * D, sC=S * D, bias=pb("proj_b"),
                   sBias=D, R=x, sR=S * D, flags=R32, wmod=wm, **kw)
            # cross-attention: q from norm2(x), k/v from y_
            self._calib_raw("dec.x2", i, x, Z)
            o.ln(x, P["ln2_g"], pb("ln2_b"), xn, S, D, Z, S * D, S * D, D, pmod=wm)
            self._calib("dec.ln2", i, xn, Z)
            w, kw = wt("q_w", D)
            o.gemm(xn, w, q, S, D, D, Z, sA=S * D, sB=D * D, sC=S * D, bias=pb("q_b"),
                   sBias=D, rope=(rt, D, S), wmod=wm, **kw)
            o.attn(q, D, S * D, kv, kv[:, :, D:], 2 * D, S * 2 * D, att, D, S * D, Z, a.dec_heads,
                   S, S)
            self._calib("dec.catt", i, att, Z)
            w, kw = wt("cproj_w", D)
            o.gemm(att, w, x, S, D, D, Z, sA=S * D, sB=D * D, sC=S * D,
                   bias=pb("cproj_b"), sBias=D, R=x, sR=S * D, flags=R32, wmod=wm, **kw)
            # MLP
            self._calib_raw("dec.x3", i, x, Z)
            o.ln(x, P["ln3_g"], pb("ln3_b"), xn, S, D, Z, S * D, S * D, D, pmod=wm)
            self._calib("dec.ln3", i, xn, Z)
            w, kw = wt("fc1_w", Dm)
            o.gemm(xn, w, hid, S, Dm, D, Z, sA=S * D, sB=Dm * D, sC=S * Dm, bias=pb("fc1_b"),
                   sBias=Dm, flags=_lib.EPI_GELU, wmod=wm, out_fp8=self.fp8, **kw)
            self._calib("dec.hid", i, hid, Z)
            w, kw = wt("fc2_w", D)
            o.gemm(hid, w, x, S, D, Dm, Z, sA=S * Dm, sB=Dm * D, sC=S * D, bias=pb("fc2_b"),
                   sBias=D, R=x, sR=S * D, flags=R32, wmod=wm, **kw)
            if (i + 1) in hook_bufs:
                hb = hook_bufs[i + 1]
                (hb if sl is None else hb[sl]).copy_(x)
                hooks[f"h{i + 1}"] = hb
                if on_hook is not None:
                    on_hook(f"h{i + 1}", hooks)
            yield i
        return hooks

    def _decode_f8fold_layer(self, i, x, xq, st, qkv, q, att, hid, hooks, hook_bufs, S, D, rt,
                             wm, sl, on_hook):
        """(Generator, one step.)  Decoder block i of _decode_folded_gen on e4m3 operands:
        the gamma-folded qkvkv / q / fc1 projections read the shifted e4m3 copy xq of x that
        the previous residual GEMM wrote (ln_stats with the calibrated shift / scale of the
        LayerNorm it feeds), attention and GELU emit e4m3, proj / cproj / fc2 run on the
        e4m3 weights with the calibrated bias shifts (_fp8_shifted_params); the hook layers'
        bf16 copies come from x directly."""
        o, a, W = self.ops, self.a, self.w
        Z = x.shape[0]
        F5, Dm = 5 * D, a.mlp_ratio * D
        P, P8, Q, F = W.dec[i], W.dec8[i], W.fp8_shift_dec[i], W.fp8_fold_dec[i]
        if sl is not None:
            P = {k: v[sl] for k, v in P.items()}
            P8 = {k: (v[0][sl], v[1][sl]) for k, v in P8.items()}
            Q = {k: v[sl] for k, v in Q.items()}
            F = {k: v[sl] for k, v in F.items()}
        last = i + 1 == a.dec_depth
        Fn = None if last else W.fp8_fold_dec[i + 1]
        if Fn is not None and sl is not None:
            Fn = {k: Fn[k][sl] for k in ("s1", "qs1")}
        R32 = dict(R=x, sR=S * D, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32)
        zs = dict(sA=S * D, sC=S * D, wmod=wm)
        tl = _tile_knob("M3S_DEC_TILE", ("qkv", "proj", "q", "cproj", "fc1", "fc2"),
                        self.dec_tiles if sl is None else self.dec_tiles_split).get
        o.gemm(xq, P8["qkvkv_wf"][0], qkv, S, F5, D, Z, sA=S * D, sB=F5 * D, sC=S * F5,
               bias=F["qkvkv_c2"], sBias=F5, rope=(rt, 3 * D, S), wmod=wm,
               ln_fold=(st, P["qkvkv_c1"], 0, F["qkvkv_c3"]), fp8=(F["qkvkv_cs"], F5),
               tile=tl("qkv"))
        o.attn(qkv, F5, S * F5, qkv[:, :, D:], qkv[:, :, 3 * D:], F5, S * F5, att,
               D, S * D, Z, a.dec_heads, S, S)
        o.gemm(att, P8["proj_w"][0], x, S, D, D, Z, sB=D * D, bias=Q["proj_b"], sBias=D,
               fp8=(P8["proj_w"][1], D), ln_stats=(xq, st, F["s2"], F["qs2"]), tile=tl("proj"),
               **zs, **R32)
        o.gemm(xq, P8["q_wf"][0], q, S, D, D, Z, sB=D * D, bias=F["q_c2"], sBias=D,
               rope=(rt, D, S), ln_fold=(st, P["q_c1"], 0, F["q_c3"]), fp8=(F["q_cs"], D),
               tile=tl("q"), **zs)
        o.attn(q, D, S * D, qkv[:, :, 2 * D:], qkv[:, :, 4 * D:], F5, S * F5, att, D,
               S * D, Z, a.dec_heads, S, S, kv_xor=1)
        o.gemm(att, P8["cproj_w"][0], x, S, D, D, Z, sB=D * D, bias=Q["cproj_b"], sBias=D,
               fp8=(P8["cproj_w"][1], D), ln_stats=(xq, st, F["s3"], F["qs3"]),
               tile=tl("cproj"), **zs, **R32)
        o.gemm(xq, P8["fc1_wf"][0], hid, S, Dm, D, Z, sA=S * D, sB=Dm * D, sC=S * Dm,
               bias=F["fc1_c2"], sBias=Dm, flags=_lib.EPI_GELU, out_fp8=True, wmod=wm,
               ln_fold=(st, P["fc1_c1"], 0, F["fc1_c3"]), fp8=(F["fc1_cs"], Dm),
               tile=tl("fc1"))
        o.gemm(hid, P8["fc2_w"][0], x, S, D, Dm, Z, sA=S * Dm, sB=Dm * D, sC=S * D,
               bias=Q["fc2_b"], sBias=D, wmod=wm, fp8=(P8["fc2_w"][1], D), tile=tl("fc2"),
               ln_stats=None if last else (xq, st, Fn["s1"], Fn["qs1"]), **R32)
        if (i + 1) in hook_bufs:
            hook_bufs[i + 1].copy_(x)
            hooks[f"h{i + 1}"] = self._buf(f"h{i + 1}", (2 * wm if sl is not None else Z,
                                                         S, D), BF16)
            if on_hook is not None:
                on_hook(f"h{i + 1}", hooks)
        yield i

    def _decode_folded(self, *args, **kw):
        return _drain(self._decode_folded_gen(*args, **kw))

    def _decode_folded_gen(self, x, xb, st, h0, Z, S, E, D, gh, gw, wm, on_hook=None, part=None):
        """(Generator: yields after issuing each block; returns the hooks.)
        decode_multi's blocks (croco/blocks.py:172-195 DecoderBlock) with every LayerNorm
        folded into the projection that consumes it (ln_fold): the residual GEMMs write x
        (f32), its bf16 copy and row statistics; qkv (norm1), the cross-attention k/v
        (norm_y of the other side), q (norm2) and fc1 (norm3) normalise in the epilogue.
        qkv of problem z and the k/v that problem z ^ 1 attends to are one GEMM over z's
        rows (PackedWeights "qkvkv"); the cross-attention reads them with kv_xor = 1.
        The hook layers' bf16 copies are written straight into the hook buffers."""
        o, a, W = self.ops, self.a, self.w
        f8f = self._f8fold()                     # e4m3 operands (xb: shifted e4m3 copy)
        adt = U8 if f8f else BF16
        F5 = 5 * D                               # fused [q | k | k' | v | v'] columns
        qkv = self._buf("dec_qkvkv", (Z, S, F5), BF16)
        q = self._buf("dec_q", (Z, S, D), BF16)
        att = self._buf("dec_att_f8" if f8f else "dec_att", (Z, S, D), adt)
        hid = self._buf("dec_hid_f8" if f8f else "dec_hid", (Z, S, a.mlp_ratio * D), adt)
        hooks = {"h0": h0}
        hook_bufs = {k: self._buf(f"h{k}", (Z, S, D), BF16) for k in a.hooks[1:3]}
        sl = None
        if part is not None:
            # one model's two problems (decode_multi's per-model split): every buffer, the
            # weight stacks and the statistics sliced to z in [2·part, 2·part + 2), weight_mod 2
            sl = slice(2 * part, 2 * part + 2)
            qkv, q, att, hid, x, xb, st = (t[sl] for t in (qkv, q, att, hid, x, xb, st))
            hook_bufs = {k: v[sl] for k, v in hook_bufs.items()}
            Z, wm = 2, 2
        rt = self.rope_tab(gh, gw)
        hk = set(a.hooks[1:3])
        Dm = a.mlp_ratio * D
        xc = xb                                  # the current bf16 copy of x
        zs = dict(sA=S * D, sC=S * D, wmod=wm)   # the per-problem strides of a [Z,S,D] A
        # tile hints (M3S_DEC_TILE experiment knob, as M3S_ENC_TILE; default: the table)
        tl = _tile_knob("M3S_DEC_TILE", ("qkv", "proj", "q", "cproj", "fc1", "fc2"),
                        self.dec_tiles if part is None else self.dec_tiles_split).get
        hot = _exp_hot_weights("dec")
        for i in range(a.dec_depth):
            P = W.dec[0 if hot else i]
            if sl is not None:
                P = {k: v[sl] for k, v in P.items()}
            R32S = dict(R=x, sR=S * D, flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32,
                        ln_stats=(xb, st))
            if f8f:
                yield from self._decode_f8fold_layer(i, x, xb, st, qkv, q, att, hid, hooks,
                                                     hook_bufs, S, D, rt, wm, sl, on_hook)
                continue
            # norm1 → qkv of problem z and norm_y → cross k/v of problem z ^ 1, one GEMM over
            # x of the layer's start (the reference's y_ = norm_y(y) before x changes)
            o.gemm(xc, P["qkvkv_wf"], qkv, S, F5, D, Z, sA=S * D, sB=F5 * D, sC=S * F5,
                   bias=P["qkvkv_c2"], sBias=F5, rope=(rt, 3 * D, S), wmod=wm,
                   ln_fold=(st, P["qkvkv_c1"], 0), tile=tl("qkv"))
            o.attn(qkv, F5, S * F5, qkv[:, :, D:], qkv[:, :, 3 * D:], F5, S * F5, att,
                   D, S * D, Z, a.dec_heads, S, S)
            o.gemm(att, P["proj_w"], x, S, D, D, Z, sB=D * D, bias=P["proj_b"], sBias=D, **zs,
                   tile=tl("proj"), **R32S)
            o.gemm(xb, P["q_wf"], q, S, D, D, Z, sB=D * D, bias=P["q_c2"], sBias=D,
                   rope=(rt, D, S), ln_fold=(st, P["q_c1"], 0), tile=tl("q"), **zs)
            # k' / v' of problem z were computed in problem z ^ 1's rows
            o.attn(q, D, S * D, qkv[:, :, 2 * D:], qkv[:, :, 4 * D:], F5, S * F5, att, D,
                   S * D, Z, a.dec_heads, S, S, kv_xor=1)
            o.gemm(att, P["cproj_w"], x, S, D, D, Z, sB=D * D, bias=P["cproj_b"], sBias=D, **zs,
                   tile=tl("cproj"), **R32S)
            o.gemm(xb, P["fc1_wf"], hid, S, Dm, D, Z, sA=S * D, sB=Dm * D, sC=S * Dm,
                   bias=P["fc1_c2"], sBias=Dm, flags=_lib.EPI_GELU, wmod=wm,
                   ln_fold=(st, P["fc1_c1"], 0), tile=tl("fc1"))
            xc = xb
            if (i + 1) in hk:
                xc = hook_bufs[i + 1]
                hooks[f"h{i + 1}"] = self._buf(f"h{i + 1}", (2 * wm if sl is not None else Z,
                                                             S, D), BF16)
            o.gemm(hid, P["fc2_w"], x, S, D, Dm, Z, sA=S * Dm, sB=Dm * D, sC=S * D,
                   bias=P["fc2_b"], sBias=D, wmod=wm, tile=tl("fc2"),
                   **dict(R32S, ln_stats=(xc, st)))
            if (i + 1) in hk and on_hook is not None:
                on_hook(f"h{i + 1}", hooks)
            yield i
        if sl is not None:
            return hooks
        h12 = self._buf("h12", (Z, S, D), BF16)
        o.ln(x, W.dec_norm_g, W.dec_norm_b, h12, S, D, Z, S * D, S * D, D, pmod=wm)
        hooks["h12"] = h12
        if on_hook is not None:
            on_hook("h12", hooks)
        return hooks

    # ---- DPT heads (batched over z) ----
    def _conv3(self, x, wkey, out, b, hin, win, cin, cout, stride=1, bias_key=None, R=None,
               flags=0, dpt=None):
        o, H = self.ops, self._hw
        hout = (hin + 2 - 3) // stride + 1
        wout = (win + 2 - 3) // stride + 1
        o.gemm(x, H(wkey), out, hout * wout, cout, 9 * cin, b, sA=hin * win * cin,
               sB=cout * 9 * cin, sC=hout * wout * cout,
               bias=H(bias_key) if bias_key else None, sBias=cout, R=R,
               sR=hout * wout * cout, flags=flags, conv=(hin, win, cin, hout, wout, stride),
               wmod=self._wm, dpt=dpt)
        return hout, wout

    def _rcu(self, x, k, u, b, h, w, out, addend_res=None):
        """ResidualConvUnit: out = conv2(relu(conv1(relu(x)))) + (x or addend_res).  The
        conv1 scratch is per unit (RCU1 runs on the aux stream beside RCU2 of the same
        resolution)."""
        F = self.a.feature_dim
        t = self._buf(("rcu_t", u, h, w), (b, h, w, F), BF16)
        self._conv3(x, f"r{k}_u{u}c1_w", t, b, h, w, F, F, bias_key=f"r{k}_u{u}c1_b",
                    flags=_lib.PRO_RELU)
        self._conv3(t, f"r{k}_u{u}c2_w", out, b, h, w, F, F, bias_key=f"r{k}_u{u}c2_b",
                    R=addend_res if addend_res is not None else x,
                    flags=_lib.PRO_RELU | _lib.EPI_RES_BF16)

    def _fusion(self, k, s1, b, h, w, next_hw, next_u, out, inv_scale=1.0):
        """FeatureFusionBlock (dpt_block.py:185-218) at resolution (h, w), from its input
        s1 = path + RCU1(skip) (refinenet4: the path alone): s = RCU2(s1);
        out = up2(out_conv(s)) + next_u — out_conv commuted before the upsample, and the
        next level's `+ RCU1(skip)` (next_u, computed ahead of this chain: `_rcu1_skip`)
        added by the upsample, so `out` is the next level's s1."""
        o, H = self.ops, self._hw
        F = self.a.feature_dim
        s2 = self._buf(("fus_s2", h, w), (b, h, w, F), BF16)
        self._rcu(s1, k, 2, b, h, w, s2)
        oc = self._buf(("fus_oc", h, w), (b, h, w, F), BF16)
        o.gemm(s2, H(f"r{k}_out_w"), oc, h * w, F, F, b, sA=h * w * F, sB=F * F, sC=h * w * F,
               bias=H(f"r{k}_out_b"), sBias=F, wmod=self._wm)
        oh, ow = next_hw
        o.up2(oc, out, b, h, w, F, oh, ow, add=next_u, inv_scale=inv_scale)

    def _rcu1_skip(self, k, skip, b, h, w):
        """refinenet k's RCU1 on its skip (layer_rn output): u = conv2(relu(conv1(relu(skip))))
        + skip.  It depends on the skip alone, so it runs beside the refinenet chain
        (`_dpt`); the chain's upsample adds it: path + RCU1(skip) is the fusion's s1."""
        F = self.a.feature_dim
        u = self._buf(("fus_u", h, w), (b, h, w, F), BF16)
        self._rcu(skip, k, 1, b, h, w, u)
        return u

    def _local_features(self, hooks, G, S, E, D, H, W):
        """MASt3R local features (z = 2, 3 of each pair): cat(enc, dec_last) → MLP → pixel
        shuffle, on side stream 1 (independent of the DPT: overlaps all of it)."""
        o, aM = self.ops, self.w.arch_mast3r
        idim = E + D
        hidd = 4 * idim
        odim = (aM.desc_dim + 1) * aM.patch ** 2
        desc = self._buf("desc", (2 * G, H, W, aM.desc_dim), F32)
        desc16 = self._buf("desc16", (2 * G, H, W, aM.desc_dim), torch.float16)
        dconf = self._buf("desc_conf", (2 * G, H, W), F32)
        with self._on(1):
            cat = self._buf("lf_cat", (2 * G, S, idim), BF16)
            # cat[g·2 + side] = [h0 | h12] of problem z = g·4 + 2 + side (MASt3R's two views)
            h0, h12 = hooks["h0"], hooks["h12"]
            if not (h0.is_contiguous() and h12.is_contiguous()):
                raise RuntimeError("local features: hooks must be contiguous")
            for src, width, off in ((h0, E, 0), (h12, D, 2 * E)):
                rb = width * 2
                o.copy_rows(src, cat, S, rb, rb, idim * 2, G, 2, 4 * S * rb, S * rb, 2 * S * rb,
                            2 * S * idim * 2, S * idim * 2, off)
            lh = self._buf("lf_hid", (2 * G, S, hidd), BF16)
            o.gemm(cat, self.w.lf_fc1_w, lh, S, hidd, idim, 2 * G, sA=S * idim,
                   sB=hidd * idim, sC=S * hidd, bias=self.w.lf_fc1_b, sBias=hidd,
                   flags=_lib.EPI_GELU, wmod=2)
            lo = self._buf("lf_out", (2 * G, S, odim), F32)
            o.gemm(lh, self.w.lf_fc2_w, lo, S, odim, hidd, 2 * G, sA=S * hidd,
                   sB=odim * hidd, sC=S * odim, bias=self.w.lf_fc2_b, sBias=odim,
                   flags=_lib.EPI_OUT_F32, wmod=2)
            o.local_features(lo, desc, desc16, dconf, 2 * G, H, W)
            ev_lf = self._event()
        return desc, desc16, dconf, ev_lf

    def _hw(self, key):
        """Head weight stack `key` from the current set's first stack (split heads)."""
        t = self.w.h[key]
        return t[self._wbase:] if self._wbase else t

    def heads(self, hooks, gh, gw, H, W, models=2, split=False):
        """DPT heads of all 2*models*G problems (z = (g*models + model)*2 + side, head weights
        z % (2*models)) + MASt3R local features of the model-1 problems (models=2 only).
        split (one pair, G = 1): the MASt3R DPT heads — whose pts3d/conf the tracking never
        reads (monst3r_utils.py:290) — are issued on side stream 0 as their own 2-problem
        set, behind the local-feature MLP (which the matching waits for) and concurrent with
        the MonST3R heads and the caller's matching / pose solve; the caller joins with
        `join()` before the next frame.
        Returns pts3d f32 [Z,H,W,3], conf f32 [Z,H,W], desc16 f16 [2G,H,W,24],
        desc f32 [2G,H,W,24], desc_conf f32 [2G,H,W] (the latter three: (g, side) of model 1;
        None with models=1)."""
        a = self.a
        Z = hooks["h0"].shape[0]
        wm = 2 * models
        G = Z // wm
        S, E, D = gh * gw, a.enc_dim, a.dec_dim
        pts = self._buf("pts3d", (Z, H, W, 3), F32)
        conf = self._buf("conf", (Z, H, W), F32)
        split = split and models == 2 and G == 1
        desc = desc16 = dconf = ev_lf = None
        if split:
            main = torch.cuda.current_stream(self.dev)
            side = self.side[0]
            side.wait_stream(main)
            # side-chain tile hints (M3S_SIDE_TILE experiment knob: lf / dpt; default table)
            st = _tile_knob("M3S_SIDE_TILE", ("lf", "dpt"), self.side_tiles)
            with torch.cuda.stream(side):
                try:
                    if self.lf_side:
                        # the local features (needed by the matching) first on the side
                        # chain, overlapping the MonST3R heads; then the MASt3R heads
                        self._wm = wm
                        self.ops.tile_default = st.get("lf")
                        desc, desc16, dconf, _ = self._local_features(hooks, G, S, E, D, H, W)
                        ev_lf = torch.cuda.Event()
                        ev_lf.record(side)
                    sub = {k: v[2:4] for k, v in hooks.items()}
                    self.ops.tile_default = st.get("dpt")
                    # M3S_ABLATE_MAST3R_DPT=1: diagnostic ablation only (tools/step_ablation):
                    # the discarded MASt3R pts3d / conf heads are not issued
                    if os.environ.get("M3S_ABLATE_MAST3R_DPT") != "1":
                        self._dpt(sub, gh, gw, H, W, 2, 2, 2, "mast3r", pts[2:4], conf[2:4])
                finally:
                    self.ops.tile_default = None
                self._ev_heads = torch.cuda.Event()
                self._ev_heads.record(side)
        # MASt3R local features (z = 2, 3): cat(enc, dec_last) → MLP → pixel shuffle
        if models == 2 and desc is None:
            self._wm = wm
            desc, desc16, dconf, ev_lf = self._local_features(hooks, G, S, E, D, H, W)
        if split:
            sub = {k: v[0:2] for k, v in hooks.items()}
            self._dpt(sub, gh, gw, H, W, 2, 0, 2, None, pts[0:2], conf[0:2])
        else:
            self._dpt(hooks, gh, gw, H, W, Z, 0, wm, None, pts, conf)
        self._wait(ev_lf)
        return pts, conf, desc16, desc, dconf

    def join(self):
        """Current stream waits for the split MASt3R heads (heads(split=True))."""
        if self._ev_heads is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._ev_heads)
            self._ev_heads = None

    def _rn_bufs(self, gh, gw, Z):
        F = self.a.feature_dim
        g3h, g3w = (gh + 1) // 2, (gw + 1) // 2
        dims = [(4 * gh, 4 * gw), (2 * gh, 2 * gw), (gh, gw), (g3h, g3w)]
        return [self._buf(f"rn{k}", (Z, dims[k][0], dims[k][1], F), BF16) for k in range(4)]

    def _ap_branch(self, k, hooks, gh, gw, Z, R):
        """DPT act_postprocess[k] + scratch.layer{k+1}_rn (d3r/heads/dpt_head.py:62-88,
        croco/dpt_block.py:300-338) of Z problems: hook → R[k] (F channels)."""
        o, a, Hw, wm = self.ops, self.a, self._hw, self._wm
        S, E, D = gh * gw, a.enc_dim, a.dec_dim
        Ld, F = a.layer_dims, a.feature_dim
        g3h, g3w = (gh + 1) // 2, (gw + 1) // 2
        if k == 0:
            t0 = self._buf("ap_t0", (Z, S, Ld[0]), BF16)
            o.gemm(hooks["h0"], Hw("ap0_w"), t0, S, Ld[0], E, Z, sA=S * E, sB=Ld[0] * E,
                   sC=S * Ld[0], bias=Hw("ap0_b"), sBias=Ld[0], wmod=wm)
            L0 = self._buf("ap_L0", (Z, 4 * gh, 4 * gw, Ld[0]), BF16)
            o.gemm(t0, Hw("ap0t_w"), L0, S, 16 * Ld[0], Ld[0], Z, sA=S * Ld[0],
                   sB=16 * Ld[0] * Ld[0], sC=16 * S * Ld[0], bias=Hw("ap0t_b"), sBias=Ld[0],
                   convt=(4, Ld[0], gw), wmod=wm)
            self._conv3(L0, "rn0_w", R[0], Z, 4 * gh, 4 * gw, Ld[0], F)
        elif k == 1:
            t1 = self._buf("ap_t1", (Z, S, Ld[1]), BF16)
            o.gemm(hooks["h6"], Hw("ap1_w"), t1, S, Ld[1], D, Z, sA=S * D, sB=Ld[1] * D,
                   sC=S * Ld[1], bias=Hw("ap1_b"), sBias=Ld[1], wmod=wm)
            L1 = self._buf("ap_L1", (Z, 2 * gh, 2 * gw, Ld[1]), BF16)
            o.gemm(t1, Hw("ap1t_w"), L1, S, 4 * Ld[1], Ld[1], Z, sA=S * Ld[1],
                   sB=4 * Ld[1] * Ld[1], sC=4 * S * Ld[1], bias=Hw("ap1t_b"), sBias=Ld[1],
                   convt=(2, Ld[1], gw), wmod=wm)
            self._conv3(L1, "rn1_w", R[1], Z, 2 * gh, 2 * gw, Ld[1], F)
        elif k == 2:
            L2 = self._buf("ap_L2", (Z, gh, gw, Ld[2]), BF16)
            o.gemm(hooks["h9"], Hw("ap2_w"), L2, S, Ld[2], D, Z, sA=S * D, sB=Ld[2] * D,
                   sC=S * Ld[2], bias=Hw("ap2_b"), sBias=Ld[2], wmod=wm)
            self._conv3(L2, "rn2_w", R[2], Z, gh, gw, Ld[2], F)
        else:
            t3 = self._buf("ap_t3", (Z, gh, gw, Ld[3]), BF16)
            o.gemm(hooks["h12"], Hw("ap3_w"), t3, S, Ld[3], D, Z, sA=S * D, sB=Ld[3] * D,
                   sC=S * Ld[3], bias=Hw("ap3_b"), sBias=Ld[3], wmod=wm)
            L3 = self._buf("ap_L3", (Z, g3h, g3w, Ld[3]), BF16)
            self._conv3(t3, "ap3c_w", L3, Z, gh, gw, Ld[3], Ld[3], stride=2, bias_key="ap3c_b")
            self._conv3(L3, "rn3_w", R[3], Z, g3h, g3w, Ld[3], F)

    def _dpt(self, hooks, gh, gw, H, W, Z, wbase, wm, tag, pts, conf):
        """act_postprocess + refinenets + head of Z problems whose hooks are given (views),
        head weights from stack wbase with weight_mod wm, scratch keyed by tag."""
        o, a = self.ops, self.a
        self._tag, self._wbase, self._wm = tag, wbase, wm
        Hw = self._hw
        F = a.feature_dim
        g3h, g3w = (gh + 1) // 2, (gw + 1) // 2
        R = self._rn_bufs(gh, gw, Z)
        # The refinenet chain needs the act_postprocess / layer_rn outputs one level at a
        # time (R[3] first, R[0] last), and each level's RCU1 depends on its skip R[k-1]
        # alone: branches 2, 1, 0, each followed by its level's RCU1 (u3, u2, u1), then
        # branch 3 and the refinenets, whose upsamples add the u's.  (The branches + RCU1s
        # on a stream of their own measured 232.6 vs 231.5 frames/s, noise, on the prefetch
        # stream the replayed step segfaulted: round 5, removed.)
        h_of = {3: (gh, gw), 2: (2 * gh, 2 * gw), 1: (4 * gh, 4 * gw)}
        u = {}
        for lvl, br in ((3, 2), (2, 1), (1, 0)):
            self._ap_branch(br, hooks, gh, gw, Z, R)
            u[lvl] = self._rcu1_skip(lvl, R[br], Z, *h_of[lvl])
        self._ap_branch(3, hooks, gh, gw, Z, R)
        # refinenets: s1_k = path_k + RCU1_k(R_{k-1}); path_{k-1} = up2(out_conv(RCU2(s1_k)))
        p4 = self._buf("path4", (Z, gh, gw, F), BF16)
        self._fusion(4, R[3], Z, g3h, g3w, (gh, gw), u[3], p4)
        p3 = self._buf("path3", (Z, 2 * gh, 2 * gw, F), BF16)
        self._fusion(3, p4, Z, gh, gw, (2 * gh, 2 * gw), u[2], p3)
        p2 = self._buf("path2", (Z, 4 * gh, 4 * gw, F), BF16)
        self._fusion(2, p3, Z, 2 * gh, 2 * gw, (4 * gh, 4 * gw), u[1], p2)
        # fp8 mode (C5): path1 and the head's upsample are emitted as e4m3 for the two
        # full-resolution convs (the others stay bf16)
        f8c = self._fp8_convs()
        inv = self.w.h8_inv
        p1 = self._buf("path1" if not f8c else "path1_e4m3", (Z, 8 * gh, 8 * gw, F),
                       U8 if f8c else BF16)
        self._fusion(1, p2, Z, 4 * gh, 4 * gw, (8 * gh, 8 * gw), None, p1,
                     inv_scale=inv.get("head0", 1.0) if f8c else 1.0)
        self._calib_amax("head0", p1)
        # head: conv3x3 F→F/2 @ (H/2, W/2), up2, conv3x3 → last_dim + ReLU, 1x1 → 4 + post
        h2, w2 = 8 * gh, 8 * gw
        hd0 = self._buf("head0", (Z, h2, w2, F // 2), BF16)
        if f8c:
            self._conv3_f8(p1, "head0", hd0, Z, h2, w2, F, F // 2, bias_key="head0_b")
        else:
            self._conv3(p1, "head0_w", hd0, Z, h2, w2, F, F // 2, bias_key="head0_b")
        hup = self._buf("head_up" if not f8c else "head_up_e4m3", (Z, H, W, F // 2),
                        U8 if f8c else BF16)
        o.up2(hd0, hup, Z, h2, w2, F // 2, H, W, inv_scale=inv.get("head2", 1.0) if f8c else 1.0)
        self._calib_amax("head2", hup)
        # conv3x3 → last_dim + ReLU with the 1x1 (last_dim → 4) + reg_dense_depth / conf
        # fused into its epilogue: the 128-channel map never reaches HBM
        dpt = (Hw("head4_w"), Hw("head4_b"), pts, conf, a.conf_min)
        if f8c:
            self._conv3_f8(hup, "head2", pts, Z, H, W, F // 2, a.last_dim, bias_key="head2_b",
                           flags=_lib.EPI_RELU, dpt=dpt)
        else:
            self._conv3(hup, "head2_w", pts, Z, H, W, F // 2, a.last_dim, bias_key="head2_b",
                        flags=_lib.EPI_RELU, dpt=dpt)
        self._tag, self._wbase = None, 0


    # ---- monst3r_asymmetric_inference ----
    def pair(self, img_i, feat_j=None, img_j=None, feat_i=None, split_heads=False):
        """Frame i vs keyframe j (keyframe features cached as in monst3r_utils.py:262-269).
        feat_i: frame i's encoder features when already computed (the prefetched encode of
        frontend.FramePipeline); img_i then only gives the size.
        Returns dict X [2,H,W,3] (ii, ji), C [2,H,W], D16 f16 [2,H,W,24], D f32, Q [2,H,W],
        feat_i (to cache when the frame becomes a keyframe).  split_heads: the MASt3R DPT
        heads (mast3r_X / mast3r_C) finish asynchronously on a side stream — call join()
        before reading them or starting the next pair."""
        a = self.a
        H, W = img_i.shape[-2:]
        gh, gw = H // a.patch, W // a.patch
        if feat_j is None:
            feat_j, _ = self.encode(img_j)
            feat_j = feat_j.clone()
        if feat_i is None:
            feat_i, pos = self.encode(img_i)
        else:
            pos = self.positions(1, gh, gw)
        hooks = self.decode(feat_i[0], feat_j.reshape(-1, a.enc_dim), pos, gh, gw)
        pts, conf, desc16, desc, dconf = self.heads(hooks, gh, gw, H, W, split=split_heads)
        return dict(X=pts[0:2], C=conf[0:2], D16=desc16, D=desc, Q=dconf, feat_i=feat_i,
                    mast3r_X=pts[2:4], mast3r_C=conf[2:4])

    # ---- one view's heads (d3r/model.py:192-196 `_downstream_head`, per model) ----
    def single_head(self, dec, model, side, H, W):
        """The heads of ONE decoded view: dec = {h0, h6, h9, h12} bf16 [1,S,*] (the decoder
        outputs at the DPT hooks, d3r/heads/dpt_head.py:110), model 0 = MonST3R (pts3d,
        conf), 1 = MASt3R (+ desc, desc_conf from the catmlp local features), side 0/1 =
        head1/head2.  Fresh tensors.  The batched pair / symmetric paths run all problems of
        a pair in one launch; this is the reference model's per-view API."""
        a = self.a
        gh, gw = H // a.patch, W // a.patch
        S, E, D = gh * gw, a.enc_dim, a.dec_dim
        tag = f"api{model}{side}"
        self._tag = tag
        pts = self._buf("api_pts", (1, H, W, 3), F32)
        conf = self._buf("api_conf", (1, H, W), F32)
        self._tag = None
        hk = {k: dec[k].reshape(1, S, -1).to(BF16).contiguous() for k in ("h0", "h6", "h9", "h12")}
        self._dpt(hk, gh, gw, H, W, 1, model * 2 + side, 1, tag, pts, conf)
        out = {"pts3d": pts.clone(), "conf": conf.clone()}
        if model == 1:
            # the local-feature MLP reads model 1 of a pair layout [model][side]: place this
            # view in both sides' slots and keep the one whose weights are this side's
            self._tag = tag
            h0 = self._buf("api_h0", (4, S, E), BF16)
            h12 = self._buf("api_h12", (4, S, D), BF16)
            h0[2:4].copy_(hk["h0"].expand(2, S, E))
            h12[2:4].copy_(hk["h12"].expand(2, S, D))
            self._wm = 4
            desc, _, dconf, ev = self._local_features({"h0": h0, "h12": h12}, 1, S, E, D, H, W)
            self._wait(ev)
            self._tag = None
            out["desc"] = desc[side:side + 1].clone()
            out["desc_conf"] = dconf[side:side + 1].clone()
        return out

    # ---- monst3r_inference_mono (monst3r_utils.py:187-211) ----
    def mono(self, feat, H, W):
        """Self-pair decode of one frame's features feat bf16 [1,S,E] by MonST3R alone (2
        problems: both sides, both heads).  Returns X [2,H,W,3] (res11, res21), C [2,H,W]
        (views of persistent buffers, overwritten by the next mono call)."""
        a = self.a
        gh, gw = H // a.patch, W // a.patch
        f = feat.reshape(1, gh * gw, a.enc_dim)
        hooks = self.decode_multi(f, f, gh, gw, models=1)
        pts, conf, _, _, _ = self.heads(hooks, gh, gw, H, W, models=1)
        return pts, conf

    # ---- monst3r_decode_symmetric_batch (monst3r_utils.py:141-184) ----
    def symmetric(self, feat_i, feat_j, H, W, chunk=None):
        """B keyframe pairs (i_b, j_b), both directions, both models.  feat_i/feat_j bf16
        [B,S,E].  The reference loops over b and runs 4 decoder calls + 8 heads per pair
        sequentially; here `chunk` pairs (8 x chunk problems) go through every launch —
        by default the B pairs in ceil(B / 7) near-equal chunks of at most 7 (round 6: at 7
        pairs the M = 768 decoder GEMMs' 256x256 tile grids end on nearly full waves —
        [768,768,768,56] 504 tiles, [768,768,3072,56] 504 — where 4 pairs left 288 tiles,
        1.1 waves).
        Returns fresh tensors in the reference's [4,B,...] order (Xii, Xji, Xjj, Xij):
        X f32 [4,B,H,W,3], C [4,B,H,W] (MonST3R), D f32 [4,B,H,W,24], D16 f16, Q [4,B,H,W]
        (MASt3R)."""
        a = self.a
        gh, gw = H // a.patch, W // a.patch
        S, E = gh * gw, a.enc_dim
        B = feat_i.shape[0]
        fi, fj = feat_i.reshape(B, S, E), feat_j.reshape(B, S, E)
        X = torch.empty((4, B, H, W, 3), dtype=F32, device=self.dev)
        C = torch.empty((4, B, H, W), dtype=F32, device=self.dev)
        D = torch.empty((4, B, H, W, 24), dtype=F32, device=self.dev)
        D16 = torch.empty((4, B, H, W, 24), dtype=torch.float16, device=self.dev)
        Q = torch.empty((4, B, H, W), dtype=F32, device=self.dev)
        if chunk is None:   # ceil(B / sym_chunk) chunks, sizes differing by at most one
            c = max(1, -(-B // self.sym_chunk))
            sizes = [B // c + (1 if i < B % c else 0) for i in range(c)]
        else:
            sizes = [min(chunk, B - b0) for b0 in range(0, B, chunk)]
        b0 = 0
        for nb in sizes:
            # directed pairs g = b*2 + d: d = 0 → (i, j), d = 1 → (j, i)
            f1 = torch.stack([fi[b0:b0 + nb], fj[b0:b0 + nb]], 1).reshape(2 * nb, S, E)
            f2 = torch.stack([fj[b0:b0 + nb], fi[b0:b0 + nb]], 1).reshape(2 * nb, S, E)
            hooks = self.decode_multi(f1, f2, gh, gw)
            pts, conf, d16, d32, dq = self.heads(hooks, gh, gw, H, W)
            # problem z = ((b*2 + d)*2 + model)*2 + side → reference slot d*2 + side
            X[:, b0:b0 + nb] = pts.view(nb, 2, 2, 2, H, W, 3)[:, :, 0].reshape(
                nb, 4, H, W, 3).transpose(0, 1)
            C[:, b0:b0 + nb] = conf.view(nb, 2, 2, 2, H, W)[:, :, 0].reshape(
                nb, 4, H, W).transpose(0, 1)
            D[:, b0:b0 + nb] = d32.view(nb, 4, H, W, 24).transpose(0, 1)
            D16[:, b0:b0 + nb] = d16.view(nb, 4, H, W, 24).transpose(0, 1)
            Q[:, b0:b0 + nb] = dq.view(nb, 4, H, W).transpose(0, 1)
            b0 += nb
        return dict(X=X, C=C, D=D, D16=D16, Q=Q)


def build(device, seed_monst3r=0, seed_mast3r=1, small=False):
    am, aM = Wt.MONST3R, Wt.MAST3R
    if small:
        am, aM = Wt.small(am), Wt.small(aM)
    sdm = Wt.make_state_dict(am, seed_monst3r)
    sdM = Wt.make_state_dict(aM, seed_mast3r)
    return PairModel(PackedWeights(sdm, am, sdM, aM, device), device), (sdm, am, sdM, aM)


def smoke(device):
    """Small-width pair inference on the GPU vs the reference goldens (tests/golden)."""
    import os

    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    g = dict(np.load(os.path.join(root, "tests", "golden", "vit_small.npz")))
    m, _ = build(device, small=True)
    t = lambda k: torch.from_numpy(g[k]).to(device)  # noqa: E731
    out = m.pair(t("img_i"), img_j=t("img_j"))
    cos = torch.nn.functional.cosine_similarity(out["D"], t("D"), dim=-1)
    rel_c = ((out["C"] - t("C")).abs() / t("C")).median()
    assert float(cos.median()) > 0.995 and float(rel_c) < 0.03, (float(cos.median()), float(rel_c))
    return float(cos.median()), float(rel_c)
