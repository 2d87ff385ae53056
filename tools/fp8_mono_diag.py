"""fp8 mono decode on the GPU against the fake-quantised restatement, stage by stage
(tools only, round 5).  tools/fp8_error_budget.py places the fp8 path's e4m3 roundings in
the fp32 restatement; this runs the HIP path (model.PairModel, fp8 on / off) on the same
512x512 frame and splits the pointmap error into encoder and decoder + head parts:
  enc   GPU features (fp8 / bf16) vs the fp32 and the fake-quant encoder (cosine)
  dec   the GPU decoder + head (fp8 / bf16) on the fp32 reference features, vs the fp32
        restatement and the fake-quant restatement of the decode on those features
Usage: python tools/fp8_mono_diag.py"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd"), os.path.join(ROOT, "tools")]
import fp8_error_budget as B  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402
from oracle import vit_ref as V  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cuda.matmul.allow_tf32 = False
S = 512


def rel(X, C, Xr, Cr):
    rx = (X.reshape(-1, 3) - Xr.reshape(-1, 3)).norm(dim=-1) / Xr.reshape(-1, 3).norm(dim=-1).clamp_min(1e-6)
    rc = (C.reshape(-1) - Cr.reshape(-1)).abs() / Cr.reshape(-1).abs()
    return f"X_med {float(rx.median()):.4f} X_p99 {float(rx.quantile(0.99)):.3f} C_med {float(rc.median()):.5f}"


def cos(a, b):
    return float(F.cosine_similarity(a.reshape(-1, a.shape[-1]).float(),
                                     b.reshape(-1, b.shape[-1]).float(), -1).median())


with torch.no_grad():
    m, (sdm, am, _, _) = Mdl.build(dev)
    sd = {k: v.to(dev) for k, v in sdm.items()}
    gen = torch.Generator(device=dev).manual_seed(9)
    img = torch.rand(1, 3, S, S, device=dev, generator=gen) * 2 - 1
    f_ref, pos = V.encode(sd, am, img)
    f_q, _ = B.encode(B.Q(["weights", "ln", "attn", "gelu"]), sd, am, img)
    X_ref, C_ref = V.inference_mono(sd, am, f_ref, pos, S, S)
    X_q, C_q = B.decode_mono(B.Q(["weights", "ln", "attn", "gelu"]), sd, am, f_ref, pos, S, S)
    X_qw, C_qw = B.decode_mono(B.Q(["weights"]), sd, am, f_ref, pos, S, S)
    print("fake-quant decode (all sites) on ref feats vs fp32:", rel(X_q, C_q, X_ref, C_ref), flush=True)
    print("fake-quant decode (weights)   on ref feats vs fp32:", rel(X_qw, C_qw, X_ref, C_ref), flush=True)
    for fp8 in (False, True):
        m.set_fp8(fp8)
        tag = "fp8 " if fp8 else "bf16"
        feat = m.encode(img)[0].clone()
        print(f"[{tag}] enc: cos vs fp32 {cos(feat, f_ref):.5f}  vs fake-quant {cos(feat, f_q):.5f}",
              flush=True)
        X, C = m.mono(f_ref[0].to(feat.dtype).contiguous(), S, S)
        X, C = X[0].clone(), C[0].clone()
        print(f"[{tag}] dec+head on ref feats: vs fp32 {rel(X, C, X_ref, C_ref)} | vs fake-quant "
              f"{rel(X, C, X_q, C_q)}", flush=True)
        X, C = m.mono(feat, S, S)
        X, C = X[0].clone(), C[0].clone()
        print(f"[{tag}] end to end: vs fp32 {rel(X, C, X_ref, C_ref)}", flush=True)
        if fp8:
            feat8 = feat
    m.set_fp8(False)
    # where the end-to-end error comes from: the fp8 encoder's features through other decoders
    X, C = m.mono(feat8, S, S)
    print(f"[bf16 dec] on fp8-encoder feats: vs fp32 {rel(X[0], C[0], X_ref, C_ref)}", flush=True)
    Xr8, Cr8 = V.inference_mono(sd, am, feat8.float().reshape(f_ref.shape), pos, S, S)
    print(f"[fp32 dec] on fp8-encoder feats: vs fp32 {rel(Xr8, Cr8, X_ref, C_ref)}", flush=True)
    Xrq, Crq = V.inference_mono(sd, am, f_q, pos, S, S)
    print(f"[fp32 dec] on fake-quant feats:  vs fp32 {rel(Xrq, Crq, X_ref, C_ref)}", flush=True)
    fb = m.encode(img)[0].clone().float().reshape(f_ref.shape)
    Xrb, Crb = V.inference_mono(sd, am, fb, pos, S, S)
    print(f"[fp32 dec] on bf16-encoder feats: vs fp32 {rel(Xrb, Crb, X_ref, C_ref)}", flush=True)
    # bias vs noise of the feature errors (per channel mean over tokens / RMS)
    for name, f in (("fp8 enc", feat8.float().reshape(f_ref.shape)), ("fake-quant", f_q),
                    ("bf16 enc", fb)):
        e = (f - f_ref)[0]
        bias = e.mean(0)
        print(f"{name:10s} feature error: rms {float(e.pow(2).mean().sqrt()):.5f}  channel-mean "
              f"rms {float(bias.pow(2).mean().sqrt()):.5f}  token-mean rms "
              f"{float(e.mean(1).pow(2).mean().sqrt()):.5f}  |f| rms "
              f"{float(f_ref.pow(2).mean().sqrt()):.4f}", flush=True)
