"""ORACLE — test infrastructure only (fp32 PyTorch reference of the floating-point path).

Functional fp32 restatement of the reference networks, driven by a state dict with the
reference's parameter names (monst3r_slam_amd/weights.py):
  PatchEmbedDust3R + enc_blocks + enc_norm   d3r/model.py:127-139, croco/blocks.py:114-130
  RoPE2D (RoPE100)                           croco/pos_embed.py:106-158 (curope kernels.cu)
  _decoder (dec_blocks / dec_blocks2)        d3r/model.py:171-190, croco/blocks.py:171-191
  DPT head                                   d3r/heads/dpt_head.py:34-65, croco/dpt_block.py
  postprocess                                d3r/heads/postprocess.py:10-58
  Cat_MLP_LocalFeatures_DPT_Pts3d            mast3r/catmlp_dpt_head.py:25-96
  monst3r_asymmetric_inference               mast3r_slam/monst3r_utils.py:255-297
Pinned against the reference's own modules by tests/golden/vit_small.npz
(tests/golden/make_vit_goldens.py).  Runs on CPU or GPU (plain torch ops).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

LN_EPS = 1e-6


def _ln(x, sd, name):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], LN_EPS)


def _lin(x, sd, name):
    return F.linear(x, sd[name + ".weight"], sd.get(name + ".bias"))


def positions(b, gh, gw, device):
    y = torch.arange(gh, device=device)
    x = torch.arange(gw, device=device)
    pos = torch.cartesian_prod(y, x).view(1, gh * gw, 2).expand(b, -1, 2).clone()
    return pos


def rope2d(tokens, pos, base=100.0):
    """tokens [B, heads, S, D]; pos [B, S, 2] (y, x)."""
    D = tokens.shape[-1] // 2
    inv_freq = 1.0 / (base ** (torch.arange(0, D, 2, device=tokens.device).float() / D))

    def rope1d(t, p):
        freqs = p.float()[:, :, None] * inv_freq[None, None]
        freqs = torch.cat((freqs, freqs), dim=-1)
        cos, sin = freqs.cos()[:, None], freqs.sin()[:, None]
        t1, t2 = t[..., :D // 2], t[..., D // 2:]
        return t * cos + torch.cat((-t2, t1), dim=-1) * sin

    y, x = tokens.chunk(2, dim=-1)
    return torch.cat((rope1d(y, pos[:, :, 0]), rope1d(x, pos[:, :, 1])), dim=-1)


def _attn(q, k, v, qpos, kpos, base):
    q = rope2d(q, qpos, base)
    k = rope2d(k, kpos, base)
    a = (q @ k.transpose(-2, -1)) * (q.shape[-1] ** -0.5)
    return a.softmax(dim=-1) @ v


def self_attention(x, pos, sd, name, heads, base):
    B, N, C = x.shape
    qkv = _lin(x, sd, name + ".qkv").reshape(B, N, 3, heads, C // heads).transpose(1, 3)
    q, k, v = [qkv[:, :, i] for i in range(3)]
    o = _attn(q, k, v, pos, pos, base).transpose(1, 2).reshape(B, N, C)
    return _lin(o, sd, name + ".proj")


def cross_attention(x, y, xpos, ypos, sd, name, heads, base):
    B, Nq, C = x.shape
    Nk = y.shape[1]
    q = _lin(x, sd, name + ".projq").reshape(B, Nq, heads, C // heads).permute(0, 2, 1, 3)
    k = _lin(y, sd, name + ".projk").reshape(B, Nk, heads, C // heads).permute(0, 2, 1, 3)
    v = _lin(y, sd, name + ".projv").reshape(B, Nk, heads, C // heads).permute(0, 2, 1, 3)
    o = _attn(q, k, v, xpos, ypos, base).transpose(1, 2).reshape(B, Nq, C)
    return _lin(o, sd, name + ".proj")


def mlp(x, sd, name):
    return _lin(F.gelu(_lin(x, sd, name + ".fc1")), sd, name + ".fc2")


def encode(sd, arch, img):
    """img [B,3,H,W] in [-1,1] → (feat [B,S,E], pos [B,S,2])."""
    B, _, H, W = img.shape
    x = F.conv2d(img, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"],
                 stride=arch.patch)
    gh, gw = x.shape[-2:]
    x = x.flatten(2).transpose(1, 2)
    pos = positions(B, gh, gw, img.device)
    for i in range(arch.enc_depth):
        p = f"enc_blocks.{i}."
        x = x + self_attention(_ln(x, sd, p + "norm1"), pos, sd, p + "attn", arch.enc_heads,
                               arch.rope_base)
        x = x + mlp(_ln(x, sd, p + "norm2"), sd, p + "mlp")
    return _ln(x, sd, "enc_norm"), pos


def decoder_block(x, y, xpos, ypos, sd, p, heads, base):
    x = x + self_attention(_ln(x, sd, p + "norm1"), xpos, sd, p + "attn", heads, base)
    y_ = _ln(y, sd, p + "norm_y")
    x = x + cross_attention(_ln(x, sd, p + "norm2"), y_, xpos, ypos, sd, p + "cross_attn",
                            heads, base)
    x = x + mlp(_ln(x, sd, p + "norm3"), sd, p + "mlp")
    return x


def decoder(sd, arch, f1, pos1, f2, pos2):
    out = [(f1, f2)]
    f1 = _lin(f1, sd, "decoder_embed")
    f2 = _lin(f2, sd, "decoder_embed")
    out.append((f1, f2))
    for i in range(arch.dec_depth):
        a, b = out[-1]
        n1 = decoder_block(a, b, pos1, pos2, sd, f"dec_blocks.{i}.", arch.dec_heads,
                           arch.rope_base)
        n2 = decoder_block(b, a, pos2, pos1, sd, f"dec_blocks2.{i}.", arch.dec_heads,
                           arch.rope_base)
        out.append((n1, n2))
    del out[1]
    out[-1] = tuple(_ln(t, sd, "dec_norm") for t in out[-1])
    dec1 = [o[0] for o in out]
    dec2 = [o[1] for o in out]
    return dec1, dec2


def _conv(x, sd, name, stride=1, padding=0):
    return F.conv2d(x, sd[name + ".weight"], sd.get(name + ".bias"), stride=stride,
                    padding=padding)


def _rcu(x, sd, p):
    out = _conv(F.relu(x), sd, p + ".conv1", padding=1)
    out = _conv(F.relu(out), sd, p + ".conv2", padding=1)
    return out + x


def _fusion(sd, p, *xs):
    out = xs[0]
    if len(xs) == 2:
        out = out + _rcu(xs[1], sd, p + ".resConfUnit1")
    out = _rcu(out, sd, p + ".resConfUnit2")
    out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    return _conv(out, sd, p + ".out_conv")


def dpt(sd, arch, prefix, tokens, H, W):
    """DPTOutputAdapter_fix.forward → [B, 4, H, W]."""
    gh, gw = H // arch.patch, W // arch.patch
    layers = [tokens[h] for h in arch.hooks]
    layers = [l.transpose(1, 2).reshape(l.shape[0], l.shape[2], gh, gw) for l in layers]
    p = prefix + ".dpt."
    ap = p + "act_postprocess."
    l0 = F.conv_transpose2d(_conv(layers[0], sd, ap + "0.0"), sd[ap + "0.1.weight"],
                            sd[ap + "0.1.bias"], stride=4)
    l1 = F.conv_transpose2d(_conv(layers[1], sd, ap + "1.0"), sd[ap + "1.1.weight"],
                            sd[ap + "1.1.bias"], stride=2)
    l2 = _conv(layers[2], sd, ap + "2.0")
    l3 = _conv(_conv(layers[3], sd, ap + "3.0"), sd, ap + "3.1", stride=2, padding=1)
    ls = [l0, l1, l2, l3]
    ls = [_conv(l, sd, p + f"scratch.layer{k + 1}_rn", padding=1) for k, l in enumerate(ls)]
    s = p + "scratch."
    path4 = _fusion(sd, s + "refinenet4", ls[3])[:, :, :ls[2].shape[2], :ls[2].shape[3]]
    path3 = _fusion(sd, s + "refinenet3", path4, ls[2])
    path2 = _fusion(sd, s + "refinenet2", path3, ls[1])
    path1 = _fusion(sd, s + "refinenet1", path2, ls[0])
    out = _conv(path1, sd, p + "head.0", padding=1)
    out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    out = F.relu(_conv(out, sd, p + "head.2", padding=1))
    return _conv(out, sd, p + "head.4")


def reg_dense_depth(xyz):
    d = xyz.norm(dim=-1, keepdim=True)
    return xyz / d.clip(min=1e-8) * torch.expm1(d)


def head(sd, arch, head_num, dec, H, W):
    """_downstream_head(head_num, dec, (H, W)) → dict (postprocessed)."""
    prefix = f"downstream_head{head_num}"
    out = dpt(sd, arch, prefix, dec, H, W)
    if arch.head == "catmlp+dpt":
        cat = torch.cat([dec[0], dec[-1]], dim=-1)
        B, S, _ = cat.shape
        lf = mlp(cat, sd, prefix + ".head_local_features")
        lf = lf.transpose(-1, -2).view(B, -1, H // arch.patch, W // arch.patch)
        lf = F.pixel_shuffle(lf, arch.patch)
        out = torch.cat([out, lf], dim=1)
    fmap = out.permute(0, 2, 3, 1)
    res = dict(pts3d=reg_dense_depth(fmap[..., 0:3]),
               conf=arch.conf_min + fmap[..., 3].exp())
    if arch.head == "catmlp+dpt":
        desc = fmap[..., 4:4 + arch.desc_dim]
        res["desc"] = desc / desc.norm(dim=-1, keepdim=True)
        res["desc_conf"] = arch.desc_conf_min + fmap[..., 4 + arch.desc_dim].exp()
    return res


@torch.no_grad()
def asymmetric_inference(sd_monst3r, a_monst3r, sd_mast3r, a_mast3r, img_i, img_j,
                         feat_j=None):
    """monst3r_utils.monst3r_asymmetric_inference (:255-297) for one pair (frame i,
    keyframe j).  Both decoders consume MonST3R encoder features.  Returns X [2,H,W,3],
    C [2,H,W], D [2,H,W,24], Q [2,H,W] (index 0 = ii, 1 = ji)."""
    H, W = img_i.shape[-2:]
    fi, pi = encode(sd_monst3r, a_monst3r, img_i)
    if feat_j is None:
        fj, pj = encode(sd_monst3r, a_monst3r, img_j)
    else:
        fj, pj = feat_j
    d1, d2 = decoder(sd_monst3r, a_monst3r, fi, pi, fj, pj)
    r11 = head(sd_monst3r, a_monst3r, 1, d1, H, W)
    r21 = head(sd_monst3r, a_monst3r, 2, d2, H, W)
    e1, e2 = decoder(sd_mast3r, a_mast3r, fi, pi, fj, pj)
    m11 = head(sd_mast3r, a_mast3r, 1, e1, H, W)
    m21 = head(sd_mast3r, a_mast3r, 2, e2, H, W)
    X = torch.stack([r11["pts3d"][0], r21["pts3d"][0]])
    C = torch.stack([r11["conf"][0], r21["conf"][0]])
    D = torch.stack([m11["desc"][0], m21["desc"][0]])
    Q = torch.stack([m11["desc_conf"][0], m21["desc_conf"][0]])
    return X, C, D, Q, (fi, pi), (fj, pj)


@torch.no_grad()
def decode_symmetric_batch(sd_monst3r, a_monst3r, sd_mast3r, a_mast3r, feat_i, pos_i, feat_j,
                           pos_j, H, W):
    """monst3r_utils.monst3r_decode_symmetric_batch (:141-184): per pair b, the MASt3R and
    MonST3R decoders on (i, j) and (j, i); returns X, C (MonST3R) and D, Q (MASt3R), each
    stacked [4, B, ...] in the order (ii, ji, jj, ij) (:155-183)."""
    X, C, D, Q = [], [], [], []
    for b in range(feat_i.shape[0]):
        f1, f2 = feat_i[b][None], feat_j[b][None]
        p1, p2 = pos_i[b][None], pos_j[b][None]
        res = []
        for (fa, pa, fb, pb) in ((f1, p1, f2, p2), (f2, p2, f1, p1)):
            e1, e2 = decoder(sd_mast3r, a_mast3r, fa, pa, fb, pb)
            res += [head(sd_mast3r, a_mast3r, 1, e1, H, W), head(sd_mast3r, a_mast3r, 2, e2, H, W)]
        D.append(torch.stack([r["desc"][0] for r in res]))
        Q.append(torch.stack([r["desc_conf"][0] for r in res]))
        res = []
        for (fa, pa, fb, pb) in ((f1, p1, f2, p2), (f2, p2, f1, p1)):
            d1, d2 = decoder(sd_monst3r, a_monst3r, fa, pa, fb, pb)
            res += [head(sd_monst3r, a_monst3r, 1, d1, H, W),
                    head(sd_monst3r, a_monst3r, 2, d2, H, W)]
        X.append(torch.stack([r["pts3d"][0] for r in res]))
        C.append(torch.stack([r["conf"][0] for r in res]))
    return (torch.stack(X, 1), torch.stack(C, 1), torch.stack(D, 1), torch.stack(Q, 1))


@torch.no_grad()
def inference_mono(sd_monst3r, a_monst3r, feat, pos, H, W):
    """monst3r_utils.monst3r_inference_mono (:187-211): self-pair MonST3R decode →
    Xii [1,N,3], Cii [1,N,1]."""
    d1, d2 = decoder(sd_monst3r, a_monst3r, feat, pos, feat, pos)
    r11 = head(sd_monst3r, a_monst3r, 1, d1, H, W)
    return r11["pts3d"].reshape(1, -1, 3), r11["conf"].reshape(1, -1, 1)
