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
