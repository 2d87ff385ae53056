"""fp8 calibration algebra on CPU (model.calibrate_fp8 / _fp8_shifted_params, DESIGN §2
"fp8 calibration"): the calibrated parameter copies move a per-channel shift mu out of each
e4m3 operand and into the biases without changing any exact pre-activation —
  LayerNorm → GEMM:   LN(x; beta - mu) W^T + (b + W mu) == LN(x; beta) W^T + b
  attention → proj:    v bias - mu shifts the attention output by -mu (softmax rows sum to
                       1); proj bias + W mu restores it
  GELU → fc2:          b - (Wq - W) mu (bias correction: E[(Wq - W) h] removed)
checked in f64 on the small architecture with random means."""
import torch

from monst3r_slam_amd import model as Mdl
from monst3r_slam_amd import weights as Wt


def _packed():
    am, aM = Wt.small(Wt.MONST3R), Wt.small(Wt.MAST3R)
    pw = Mdl.PackedWeights(Wt.make_state_dict(am, 0), am, Wt.make_state_dict(aM, 1), aM, "cpu")
    pw.enable_fp8()
    return pw


def _cal(pw, g):
    L, E = pw.arch.enc_depth, pw.arch.enc_dim
    D, Dm = pw.arch.dec_dim, pw.arch.dec_dim * pw.arch.mlp_ratio
    cal = {}
    for i in range(L):
        for site, n in (("enc.ln1", E), ("enc.att", E), ("enc.ln2", E),
                        ("enc.hid", E * pw.arch.mlp_ratio)):
            cal[(site, i)] = torch.randn(n, generator=g, dtype=torch.float64)
    for i in range(len(pw.dec)):
        for site, n in (("dec.ln1", D), ("dec.att", D), ("dec.lny", D), ("dec.ln2", D),
                        ("dec.catt", D), ("dec.ln3", D), ("dec.hid", Dm)):
            cal[(site, i)] = torch.randn(4, n, generator=g, dtype=torch.float64)
    return cal


def test_shifted_params_preserve_preactivations():
    pw = _packed()
    g = torch.Generator().manual_seed(0)
    cal = _cal(pw, g)
    enc, dec = Mdl._fp8_shifted_params(pw, cal)
    f64 = torch.float64
    P = pw.enc
    E = pw.arch.enc_dim
    i = 1
    x = torch.randn(5, E, generator=g, dtype=f64)          # a normalised LN output (γ x̂)
    mu = cal[("enc.ln1", i)]
    W, b = P["qkv_w"][i].to(f64), P["qkv_b"][i].to(f64)
    ref = (x + P["ln1_b"][i].to(f64)) @ W.t() + b
    got = (x + enc["ln1_b"][i].to(f64)) @ W.t() + enc["qkv_b"][i].to(f64)
    got[:, 2 * E:] += cal[("enc.att", i)]                  # the v columns carry -mu_att
    assert torch.allclose(got, ref, rtol=0, atol=1e-4 * float(ref.abs().max()))
    # proj: output of attention o; the shifted path sees o - mu_att
    o = torch.randn(5, E, generator=g, dtype=f64)
    ma = cal[("enc.att", i)]
    Wp = P["proj_w"][i].to(f64)
    ref = o @ Wp.t() + P["proj_b"][i].to(f64)
    got = (o - ma) @ Wp.t() + enc["proj_b"][i].to(f64)
    assert torch.allclose(got, ref, rtol=0, atol=1e-4 * float(ref.abs().max()))
    # fc2: bias correction with the quantised rows
    q, sc = pw.enc8["fc2_w"]
    Wq = q[i].view(torch.float8_e4m3fn).to(f64) * sc[i].to(f64)[:, None]
    W2 = P["fc2_w"][i].to(f64)
    mh = cal[("enc.hid", i)]
    corr = enc["fc2_b"][i].to(f64) - P["fc2_b"][i].to(f64)
    assert torch.allclose(corr, -(Wq - W2) @ mh, rtol=1e-5, atol=1e-6)
    # decoder, problem z = 3 (MASt3R side 2): the cross-attention k / v projection of norm_y
    D = pw.arch.dec_dim
    Pd, z, li = pw.dec[0], 3, 0
    y = torch.randn(5, D, generator=g, dtype=f64)
    my, mc = cal[("dec.lny", li)][z], cal[("dec.catt", li)][z]
    Wkv, bkv = Pd["kv_w"][z].to(f64), Pd["kv_b"][z].to(f64)
    ref = (y + Pd["lny_b"][z].to(f64)) @ Wkv.t() + bkv
    got = (y + dec[li]["lny_b"][z].to(f64)) @ Wkv.t() + dec[li]["kv_b"][z].to(f64)
    got[:, D:] += mc
    assert torch.allclose(got, ref, rtol=0, atol=1e-4 * float(ref.abs().max()))
    for k, v in list(enc.items()) + [kv for d in dec for kv in d.items()]:
        assert v.dtype == torch.float32 and v.is_contiguous(), k


def _raw(pw, g):
    """Calibrated raw residual-stream statistics (mean, max, min) per LayerNorm site."""
    L, E, D = pw.arch.enc_depth, pw.arch.enc_dim, pw.arch.dec_dim
    raw = {}

    def stats(*shape):
        m = torch.randn(*shape, generator=g, dtype=torch.float64)
        return (m, m + 1 + torch.rand(*shape, generator=g, dtype=torch.float64),
                m - 1 - torch.rand(*shape, generator=g, dtype=torch.float64))
    for i in range(L):
        for site in ("enc.x1", "enc.x2"):
            raw[(site, i)] = stats(E)
    for i in range(len(pw.dec)):
        for site in ("dec.x1", "dec.x2", "dec.x3"):
            raw[(site, i)] = stats(4, D)
    return raw


def test_fold_params_reproduce_layernorm_projection():
    """fp8 LayerNorm fold (round 6, _fp8_fold_params): with the shifted, scaled copy
    A = (x − s)·q (no e4m3 rounding here), B = W'/sw, col_scale = sw / q, c3 = W's and the
    epilogue rstd (A·Bᵀ·col_scale + c3 − mean·c1) + c2, the consumer computes exactly
    LN(x; γ, β)·Wᵀ + b — minus the attention-output shift on the v columns that the
    LayerNorm path's calibrated bias also carries.  q = 448 / (2 max |x − s|)."""
    pw = _packed()
    g = torch.Generator().manual_seed(1)
    cal, raw = _cal(pw, g), _raw(pw, g)
    enc, dec = Mdl._fp8_fold_params(pw, cal, raw)
    f64 = torch.float64
    P, E, i = pw.enc, pw.arch.enc_dim, 1
    x = torch.randn(6, E, generator=g, dtype=f64) * 3 + 2
    s, q = enc["s1"][i].to(f64), enc["qs1"][i].to(f64)
    mean, mx, mn = raw[("enc.x1", i)]
    assert torch.allclose(q, 448.0 / (2.0 * torch.maximum(mx - mean, mean - mn).max()))
    sw = pw.enc8["qkv_wf"][1][i].to(f64)
    wf = P["qkv_wf"][i].to(f64)
    A = (x - s) * q
    acc = A @ (wf / sw[:, None]).t() * enc["qkv_cs"][i].to(f64) + enc["qkv_c3"][i].to(f64)
    mu = x.mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(((x - mu) ** 2).mean(-1, keepdim=True) + Mdl.LN_EPS)
    got = rstd * (acc - mu * P["qkv_c1"][i].to(f64)) + enc["qkv_c2"][i].to(f64)
    got[:, 2 * E:] += cal[("enc.att", i)]
    ln = torch.nn.functional.layer_norm(x, (E,), P["ln1_g"][i].to(f64), P["ln1_b"][i].to(f64),
                                        eps=Mdl.LN_EPS)
    ref = ln @ P["qkv_w"][i].to(f64).t() + P["qkv_b"][i].to(f64)
    # (W' = bf16(W∘γ): the reference uses the bf16-rounded fold too)
    ref_f = rstd * ((x - mu) @ wf.t()) + P["qkv_c2"][i].to(f64)
    # (the parameters are stored in f32: 1e-5 of the output scale)
    assert torch.allclose(got, ref_f, rtol=0, atol=1e-5 * float(ref_f.abs().max()))
    assert torch.allclose(got, ref, rtol=0, atol=2e-2 * float(ref.abs().max()))
    # decoder: the fused [q | k | k' | v | v'] bias carries this problem's self-attention
    # shift on v and problem z ^ 1's cross-attention shift on v'
    D, d0 = pw.arch.dec_dim, dec[0]
    c2 = pw.dec[0]["qkvkv_c2"].to(f64)
    assert torch.allclose(d0["qkvkv_c2"].to(f64)[:, 3 * D:4 * D],
                          (c2[:, 3 * D:4 * D] - cal[("dec.att", 0)]).float().to(f64))
    assert torch.allclose(d0["qkvkv_c2"].to(f64)[:, 4 * D:],
                          (c2[:, 4 * D:] - cal[("dec.catt", 0)][[1, 0, 3, 2]]).float().to(f64))
    assert d0["qs1"].shape == (4,) and d0["s2"].shape == (4, D)


def test_epilogue_bytes_counts_stored_operands():
    """bench._epilogue_bytes: a residual GEMM with LayerNorm statistics and the bf16 copy
    reads A, B (bf16), reads and writes the f32 residual, writes the copy and 8 B of
    statistics per 128 columns; the e4m3 copy is one byte; an implicit conv reads its image
    once (M·K/9); the fused DPT tail writes 16 B per row instead of C."""
    import bench
    from monst3r_slam_amd import _lib
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.batch = 768, 768, 3072, 2
    d.flags = _lib.EPI_OUT_F32 | _lib.EPI_RES_F32 | _lib.EPI_LN_STATS | _lib.EPI_BIAS
    per = (768 * 3072 + 768 * 3072) * 2 + 768 * 768 * 4 * 2 + 768 * 768 * 2 + 768 * 6 * 8
    assert bench._epilogue_bytes(d) == 2 * per
    buf = torch.zeros(1)
    d.ln_shift = buf.data_ptr()
    assert bench._epilogue_bytes(d) == 2 * (per - 768 * 768)
    c = _lib.GemmDesc()
    c.M, c.N, c.K, c.batch, c.mode = 196608, 128, 1152, 1, 1
    c.flags = _lib.EPI_DPT_OUT | _lib.EPI_RELU | _lib.EPI_BIAS
    assert bench._epilogue_bytes(c) == (196608 * 128 + 128 * 1152) * 2 + 196608 * 16
