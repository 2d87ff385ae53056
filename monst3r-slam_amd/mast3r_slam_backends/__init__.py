"""Drop-in replacement for the reference's native module ``mast3r_slam_backends``.

Same five entry points, argument order, dtypes and return lists as the pybind11 module
built from mast3r_slam/backend (gn.cpp:116-122, gn.h:89-117), so mast3r_slam/matching.py
(:60,:79) and global_opt2.py (:148,:198) run unmodified with this directory on sys.path.
Behind them: the MI355X HIP kernels of libmonst3r_slam_amd.so via its C ABI.

Conventions kept from the reference:
  * inputs are borrowed tensors; outputs freshly allocated zeros in the input's options;
  * non-contiguous inputs raise RuntimeError("<name> must be contiguous");
  * gauss_newton_* update ``Twc`` in place and return ``[dx]``; a failed Cholesky gives a
    zero step (gn_kernels.cu:142-150).
Differences (no effect on results): kernels run on torch's current stream (the reference
used the legacy default stream), any n is accepted (no n % 16 == 0 requirement), and the
GN solve runs on the GPU in fp64 with no per-iteration host round trip.
"""
from __future__ import annotations

import os
import sys

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

from monst3r_slam_amd import _lib  # noqa: E402

__all__ = ["iter_proj", "refine_matches", "gauss_newton_rays", "gauss_newton_calib",
           "gauss_newton_points"]


def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh):
    """gn.cpp:84-99 / matching_kernels.cu:279-316."""
    _lib.require_contiguous(rays_img_with_grad=rays_img_with_grad, pts_3d_norm=pts_3d_norm,
                            p_init=p_init)
    _lib.require_cuda(rays_img_with_grad, pts_3d_norm, p_init,
                      names=("rays_img_with_grad", "pts_3d_norm", "p_init"))
    b, h, w, c = rays_img_with_grad.shape
    if c != 9:
        raise RuntimeError("rays_img_with_grad must have 9 channels (ray, d/dx, d/dy)")
    n = p_init.shape[1]
    p_new = torch.zeros((b, n, 2), dtype=p_init.dtype, device=p_init.device)
    converged = torch.zeros((b, n), dtype=torch.bool, device=p_init.device)
    st = _lib.load().m3s_iter_proj(
        _lib.ptr(rays_img_with_grad.float()), _lib.ptr(pts_3d_norm.float()),
        _lib.ptr(p_init.float()), _lib.ptr(p_new), _lib.ptr(converged), b, h, w, n,
        int(max_iter), float(lambda_init), float(cost_thresh), _lib.stream(p_init.device))
    _lib.check(st, "iter_proj")
    return [p_new, converged]


def refine_matches(D11, D21, p1, window_size, dilation_max):
    """gn.cpp:101-114 / matching_kernels.cu:84-116 (half descriptors, as matching.py:79-85
    passes them)."""
    _lib.require_contiguous(D11=D11, D21=D21, p1=p1)
    _lib.require_cuda(D11, D21, p1, names=("D11", "D21", "p1"))
    if D11.dtype != torch.float16 or D21.dtype != torch.float16:
        raise RuntimeError("refine_matches: D11/D21 must be float16 (matching.py passes .half())")
    if p1.dtype != torch.int64:
        raise RuntimeError("refine_matches: p1 must be int64")
    b, h, w, f = D11.shape
    n = p1.shape[1]
    p1_new = torch.zeros((b, n, 2), dtype=p1.dtype, device=p1.device)
    st = _lib.load().m3s_refine_matches(
        _lib.ptr(D11), _lib.ptr(D21), _lib.ptr(p1), _lib.ptr(p1_new), b, h, w, n, f,
        int(window_size), int(dilation_max), _lib.stream(p1.device))
    _lib.check(st, "refine_matches")
    return [p1_new]


def _gn_common(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q):
    _lib.require_contiguous(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx_ii2jj=idx_ii2jj,
                            valid_match=valid_match, Q=Q)
    _lib.require_cuda(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q,
                      names=("Twc", "Xs", "Cs", "ii", "jj", "idx_ii2jj", "valid_match", "Q"))
    P, N = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    dev = Twc.device
    dx = torch.zeros((max(P - 1, 0), 7), dtype=torch.float32, device=dev)
    nbytes = _lib.load().m3s_gn_workspace_bytes(P, E, N)
    ws = torch.empty((nbytes,), dtype=torch.uint8, device=dev)
    return P, N, E, dx, ws


def _finish(status, h_status, what):
    _lib.check(status, what)
    if h_status.value == -1:  # |unique(ii ∪ jj)| != Xs.size(0)
        raise RuntimeError(f"{what}: the number of unique keyframes in ii/jj must equal "
                           "Xs.size(0)")
    # M3S_ERR_NOT_PD (-4): reference semantics — zero step, no exception


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist,
                      C_thresh, Q_thresh, max_iter, delta_thresh):
    """gn.cpp:28-50 / gn_kernels.cu:1140-1228.  Twc is updated in place."""
    import ctypes
    P, N, E, dx, ws = _gn_common(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q)
    hs = ctypes.c_int(0)
    st = _lib.load().m3s_gauss_newton_rays(
        _lib.ptr(Twc), _lib.ptr(Xs), _lib.ptr(Cs), _lib.ptr(ii), _lib.ptr(jj),
        _lib.ptr(idx_ii2jj), _lib.ptr(valid_match), _lib.ptr(Q), P, N, E, float(sigma_ray),
        float(sigma_dist), float(C_thresh), float(Q_thresh), int(max_iter), float(delta_thresh),
        _lib.ptr(dx), _lib.ptr(ws), ctypes.byref(hs), _lib.stream(Twc.device))
    _finish(st, hs, "gauss_newton_rays")
    return [dx]


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width,
                       pixel_border, z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh,
                       max_iter, delta_thresh):
    """gn.cpp:52-82 / gn_kernels.cu:1546-1638.  Twc is updated in place."""
    import ctypes
    _lib.require_contiguous(K=K)
    P, N, E, dx, ws = _gn_common(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q)
    K = K.float().contiguous()
    hs = ctypes.c_int(0)
    st = _lib.load().m3s_gauss_newton_calib(
        _lib.ptr(Twc), _lib.ptr(Xs), _lib.ptr(Cs), _lib.ptr(K), _lib.ptr(ii), _lib.ptr(jj),
        _lib.ptr(idx_ii2jj), _lib.ptr(valid_match), _lib.ptr(Q), P, N, E, int(height),
        int(width), int(pixel_border), float(z_eps), float(sigma_pixel), float(sigma_depth),
        float(C_thresh), float(Q_thresh), int(max_iter), float(delta_thresh), _lib.ptr(dx),
        _lib.ptr(ws), ctypes.byref(hs), _lib.stream(Twc.device))
    _finish(st, hs, "gauss_newton_calib")
    return [dx]


def gauss_newton_points(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_point, C_thresh,
                        Q_thresh, max_iter, delta_thresh):
    """gn.cpp:3-26 / gn_kernels.cu:725-811.  Twc is updated in place."""
    import ctypes
    P, N, E, dx, ws = _gn_common(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q)
    hs = ctypes.c_int(0)
    st = _lib.load().m3s_gauss_newton_points(
        _lib.ptr(Twc), _lib.ptr(Xs), _lib.ptr(Cs), _lib.ptr(ii), _lib.ptr(jj),
        _lib.ptr(idx_ii2jj), _lib.ptr(valid_match), _lib.ptr(Q), P, N, E, float(sigma_point),
        float(C_thresh), float(Q_thresh), int(max_iter), float(delta_thresh), _lib.ptr(dx),
        _lib.ptr(ws), ctypes.byref(hs), _lib.stream(Twc.device))
    _finish(st, hs, "gauss_newton_points")
    return [dx]
