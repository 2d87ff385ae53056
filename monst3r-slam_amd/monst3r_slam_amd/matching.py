"""Projective matching — mirror of mast3r_slam/matching.py (match :8-10,
match_iterative_proj :52-90, pixel_to_lin :13-15, lin_to_pixel :18-22,
prep_for_iter_proj :25-49) over the fused HIP kernels:

  m3s_match_prep      normalise + Scharr gradient + p_init   (replaces ~5 torch passes)
  m3s_iter_proj       LM projective search (10 iterations per pixel)
  m3s_match_occlusion trunc + 3-D distance test
  m3s_refine_matches  dilated f16 descriptor argmax
  m3s_pixel_to_lin    linear index
"""
from __future__ import annotations

import torch

from . import _lib
from .config import config as _config

def pixel_to_lin(p1, w):
    return p1[..., 0] + (w * p1[..., 1])


def lin_to_pixel(idx_1_to_2, w):
    return torch.stack((idx_1_to_2 % w, idx_1_to_2 // w), dim=-1)


def prep_for_iter_proj(X11, X21, idx_1_to_2_init=None):
    """matching.py:25-49 → (rays_with_grad [b,h,w,9], pts3d_norm [b,hw,3], p_init [b,hw,2])."""
    X11 = X11.float().contiguous()
    X21 = X21.float().contiguous()
    b, h, w, _ = X11.shape
    dev = X11.device
    rwg = torch.empty((b, h, w, 9), dtype=torch.float32, device=dev)
    pts = torch.empty((b, h * w, 3), dtype=torch.float32, device=dev)
    p_init = torch.empty((b, h * w, 2), dtype=torch.float32, device=dev)
    idx = None if idx_1_to_2_init is None else idx_1_to_2_init.to(torch.int64).contiguous()
    st = _lib.load().m3s_match_prep(_lib.ptr(X11), _lib.ptr(X21), _lib.ptr(idx), _lib.ptr(rwg),
                                    _lib.ptr(pts), _lib.ptr(p_init), b, h, w, _lib.stream(dev))
    _lib.check(st, "match_prep")
    return rwg, pts, p_init


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=None, idx_out=None):
    """matching.py:52-90.  Returns (idx_1_to_2 [b,hw] int64, valid [b,hw,1] bool).
    idx_out: int64 [b,hw] to write the indices into (may be idx_1_to_2_init itself: the
    kernels read the seed before the last one writes the result, in stream order)."""
    cfg = cfg or _config["matching"]
    _lib.require_cuda(X11, X21, D11, D21, names=("X11", "X21", "D11", "D21"))
    lib = _lib.load()
    X11 = X11.float().contiguous()
    X21 = X21.float().contiguous()
    b, h, w = X21.shape[:3]
    n = h * w
    dev = X11.device
    s = _lib.stream(dev)
    rwg, pts, p_init = prep_for_iter_proj(X11, X21, idx_1_to_2_init)
    p = torch.empty((b, n, 2), dtype=torch.float32, device=dev)
    conv = torch.empty((b, n), dtype=torch.uint8, device=dev)
    # cfg["iter_proj_fma"] (opt-in): the FMA-contracted numeric model of the reference
    # binary's nvcc --fmad=true build instead of its source taken literally
    ip = lib.m3s_iter_proj_fma if cfg.get("iter_proj_fma", False) else lib.m3s_iter_proj
    _lib.check(ip(_lib.ptr(rwg), _lib.ptr(pts), _lib.ptr(p_init), _lib.ptr(p), _lib.ptr(conv), b,
                  h, w, n, int(cfg["max_iter"]), float(cfg["lambda_init"]),
                  float(cfg["convergence_thresh"]), s), "iter_proj")
    p1 = torch.empty((b, n, 2), dtype=torch.int64, device=dev)
    valid = torch.empty((b, n), dtype=torch.uint8, device=dev)
    _lib.check(lib.m3s_match_occlusion(_lib.ptr(X11), _lib.ptr(X21), _lib.ptr(p), _lib.ptr(conv),
                                       _lib.ptr(p1), _lib.ptr(valid), b, h, w,
                                       float(cfg["dist_thresh"]), s), "match_occlusion")
    if cfg["radius"] > 0:
        d11 = D11.half().contiguous()
        d21 = D21.reshape(b, n, -1).half().contiguous()
        p1n = torch.empty_like(p1)
        _lib.check(lib.m3s_refine_matches(_lib.ptr(d11), _lib.ptr(d21), _lib.ptr(p1),
                                          _lib.ptr(p1n), b, h, w, n, d11.shape[-1],
                                          int(cfg["radius"]), int(cfg["dilation_max"]), s),
                   "refine_matches")
        p1 = p1n
    if idx_out is not None:
        if idx_out.shape != (b, n) or idx_out.dtype != torch.int64 or not idx_out.is_contiguous():
            raise RuntimeError("match: idx_out must be contiguous int64 [b, h*w]")
        idx = idx_out
    else:
        idx = torch.empty((b, n), dtype=torch.int64, device=dev)
    _lib.check(lib.m3s_pixel_to_lin(_lib.ptr(p1), _lib.ptr(idx), b, n, w, s), "pixel_to_lin")
    # the kernels store 0 / 1 bytes: reinterpret as bool (no conversion pass)
    return idx, valid.view(torch.bool).unsqueeze(-1)


def match(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=None, idx_out=None):
    """matching.py:8-10."""
    return match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init, cfg, idx_out)
