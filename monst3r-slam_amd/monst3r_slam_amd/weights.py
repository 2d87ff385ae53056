"""Architectures and seeded random weights with the reference's parameter names.

No checkpoints exist offline, so parity and timing use deterministic
random weights generated here.  The state dicts use exactly the key names of the
reference modules, so `load_state_dict(strict=True)` into the reference models
(d3r/model.py AsymmetricCroCo3DStereo, mast3r/model.py AsymmetricMASt3R) succeeds; the
golden generator (tests/golden/make_vit_goldens.py) relies on that.

Architectures (logged constructors, out/run_main_monster_slam_26155.out:27,32):
  MonST3R: enc 1024/24/16, dec 768/12/12, RoPE100, head 'dpt', out 'pts3d',
           depth_mode ('exp',-inf,inf), conf_mode ('exp',1,inf)
  MASt3R:  same trunk, head 'catmlp+dpt', out 'pts3d+desc24', two_confs=True,
           desc_conf_mode ('exp',0,inf)
"""
from __future__ import annotations

import dataclasses
import hashlib

import numpy as np
import torch


@dataclasses.dataclass(frozen=True)
class Arch:
    enc_dim: int = 1024
    enc_depth: int = 24
    enc_heads: int = 16
    dec_dim: int = 768
    dec_depth: int = 12
    dec_heads: int = 12
    mlp_ratio: int = 4
    patch: int = 16
    head: str = "dpt"            # 'dpt' (MonST3R) or 'catmlp+dpt' (MASt3R)
    desc_dim: int = 24
    two_confs: bool = True
    conf_min: float = 1.0        # conf_mode ('exp', 1, inf)
    desc_conf_min: float = 0.0   # desc_conf_mode ('exp', 0, inf)
    feature_dim: int = 256
    last_dim: int = 128
    layer_dims: tuple = (96, 192, 384, 768)
    rope_base: float = 100.0

    @property
    def hooks(self):
        l2 = self.dec_depth
        return [0, l2 * 2 // 4, l2 * 3 // 4, l2]

    @property
    def dpt_nch(self):
        return 4  # 3 (pts3d) + 1 (conf)


MONST3R = Arch(head="dpt")
MAST3R = Arch(head="catmlp+dpt")


def small(arch: Arch) -> Arch:
    """Reduced-width, same-topology variant for CPU goldens (depths kept: the DPT hooks
    need dec_depth > 9, dpt_head.py:100); head dim stays 64."""
    return dataclasses.replace(arch, enc_dim=256, enc_heads=4, dec_dim=192, dec_heads=3)


def param_shapes(a: Arch) -> dict:
    """name -> (shape, kind) with kind in {linear_w, bias, ln_w, ln_b, conv_w, conv_b,
    convt_w, token}."""
    P = {}

    def lin(name, out_f, in_f, bias=True):
        P[name + ".weight"] = ((out_f, in_f), "linear_w")
        if bias:
            P[name + ".bias"] = ((out_f,), "bias")

    def ln(name, d):
        P[name + ".weight"] = ((d,), "ln_w")
        P[name + ".bias"] = ((d,), "ln_b")

    def conv(name, cout, cin, k, bias=True):
        P[name + ".weight"] = ((cout, cin, k, k), "conv_w")
        if bias:
            P[name + ".bias"] = ((cout,), "conv_b")

    def convt(name, cin, cout, k):
        P[name + ".weight"] = ((cin, cout, k, k), "convt_w")
        P[name + ".bias"] = ((cout,), "conv_b")

    E, D = a.enc_dim, a.dec_dim
    conv("patch_embed.proj", E, 3, a.patch)
    P["mask_token"] = ((1, 1, D), "token")
    for i in range(a.enc_depth):
        p = f"enc_blocks.{i}."
        ln(p + "norm1", E)
        lin(p + "attn.qkv", 3 * E, E)
        lin(p + "attn.proj", E, E)
        ln(p + "norm2", E)
        lin(p + "mlp.fc1", a.mlp_ratio * E, E)
        lin(p + "mlp.fc2", E, a.mlp_ratio * E)
    ln("enc_norm", E)
    lin("decoder_embed", D, E)
    for blocks in ("dec_blocks", "dec_blocks2"):
        for i in range(a.dec_depth):
            p = f"{blocks}.{i}."
            ln(p + "norm1", D)
            lin(p + "attn.qkv", 3 * D, D)
            lin(p + "attn.proj", D, D)
            lin(p + "cross_attn.projq", D, D)
            lin(p + "cross_attn.projk", D, D)
            lin(p + "cross_attn.projv", D, D)
            lin(p + "cross_attn.proj", D, D)
            ln(p + "norm2", D)
            ln(p + "norm3", D)
            lin(p + "mlp.fc1", a.mlp_ratio * D, D)
            lin(p + "mlp.fc2", D, a.mlp_ratio * D)
            ln(p + "norm_y", D)
    ln("dec_norm", D)
    dims = [E, D, D, D]
    L = a.layer_dims
    F = a.feature_dim
    for h in ("downstream_head1", "downstream_head2"):
        p = h + ".dpt."
        conv(p + "act_postprocess.0.0", L[0], dims[0], 1)
        convt(p + "act_postprocess.0.1", L[0], L[0], 4)
        conv(p + "act_postprocess.1.0", L[1], dims[1], 1)
        convt(p + "act_postprocess.1.1", L[1], L[1], 2)
        conv(p + "act_postprocess.2.0", L[2], dims[2], 1)
        conv(p + "act_postprocess.3.0", L[3], dims[3], 1)
        conv(p + "act_postprocess.3.1", L[3], L[3], 3)
        for k in range(4):
            conv(p + f"scratch.layer{k + 1}_rn", F, L[k], 3, bias=False)
        for k in range(1, 5):
            q = p + f"scratch.refinenet{k}."
            conv(q + "out_conv", F, F, 1)
            for u in ("resConfUnit1", "resConfUnit2"):
                conv(q + u + ".conv1", F, F, 3)
                conv(q + u + ".conv2", F, F, 3)
        conv(p + "head.0", F // 2, F, 3)
        conv(p + "head.2", a.last_dim, F // 2, 3)
        conv(p + "head.4", a.dpt_nch, a.last_dim, 1)
        if a.head == "catmlp+dpt":
            idim = E + D
            hid = 4 * idim
            odim = (a.desc_dim + int(a.two_confs)) * a.patch ** 2
            lin(h + ".head_local_features.fc1", hid, idim)
            lin(h + ".head_local_features.fc2", odim, hid)
    return P


def _seed(name: str, seed: int) -> int:
    return int.from_bytes(hashlib.sha256(f"{seed}:{name}".encode()).digest()[:8], "little")


def _draw(shape, kind, rng):
    if kind == "linear_w":
        fo, fi = shape
        b = np.sqrt(6.0 / (fi + fo))
        return rng.uniform(-b, b, size=shape)
    if kind == "bias":
        return rng.uniform(-0.02, 0.02, size=shape)
    if kind == "ln_w":
        return 1.0 + rng.uniform(-0.05, 0.05, size=shape)
    if kind == "ln_b":
        return rng.uniform(-0.02, 0.02, size=shape)
    if kind == "conv_w":
        fan_in = shape[1] * shape[2] * shape[3]
        b = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-b, b, size=shape)
    if kind == "convt_w":
        fan_in = shape[1] * shape[2] * shape[3]
        b = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-b, b, size=shape)
    if kind == "conv_b":
        return rng.uniform(-0.05, 0.05, size=shape)
    if kind == "token":
        return rng.normal(0, 0.02, size=shape)
    raise ValueError(kind)


def make_state_dict(arch: Arch, seed: int = 0, device="cpu") -> dict:
    """Deterministic (platform-independent numpy PCG64) f32 weights, reference key names.
    Includes the DPT `scratch.layer_rn.{k}` aliases of `scratch.layer{k+1}_rn`."""
    sd = {}
    for name, (shape, kind) in param_shapes(arch).items():
        rng = np.random.default_rng(_seed(name, seed))
        sd[name] = torch.from_numpy(_draw(shape, kind, rng).astype(np.float32)).to(device)
    for h in ("downstream_head1", "downstream_head2"):
        for k in range(4):
            sd[f"{h}.dpt.scratch.layer_rn.{k}.weight"] = sd[f"{h}.dpt.scratch.layer{k + 1}_rn.weight"]
    return sd


def num_params(arch: Arch) -> int:
    return int(sum(np.prod(s) for s, _ in param_shapes(arch).values()))
