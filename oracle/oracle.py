"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline, never as the thing measured or shipped.

Python side of the CPU restatement of the reference's matching / GN path:
  * ctypes bindings of oracle/_build/liboracle.so (matching_ref.c, gn_ref.c);
  * numpy restatements of the reference's Python prep (matching.py:8-90, image.py:5-38).
Reference citations are to /root/reference/MASt3R-SLAM/mast3r_slam/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.ref_iter_proj.argtypes = [P, P, P, P, P, i64, i64, i64, i64, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_float, ctypes.c_float]
        L.ref_iter_proj.restype = None
        L.ref_iter_proj_fma.argtypes = L.ref_iter_proj.argtypes
        L.ref_iter_proj_fma.restype = None
        L.ref_refine_matches.argtypes = [P, P, P, P, i64, i64, i64, i64, i64, ctypes.c_int,
                                         ctypes.c_int]
        L.ref_refine_matches.restype = None
        L.ref_gauss_newton.argtypes = [P, P, P, P, P, P, P, P, P, i64, i64, i64, ctypes.c_int,
                                       ctypes.c_float, P, P, P, P]
        L.ref_gauss_newton.restype = ctypes.c_int
        L.ref_retr_sim3.argtypes = [P, P, P]
        L.ref_rel_sim3.argtypes = [P, P, P]
        L.ref_match_prep.argtypes = [P, P, P, P, P, P, i64, i64, i64]
        L.ref_match_prep.restype = None
        L.ref_match_occlusion.argtypes = [P, P, P, P, P, P, i64, i64, i64, ctypes.c_float]
        L.ref_match_occlusion.restype = None
        L.ref_float_to_half.argtypes = [ctypes.c_float]
        L.ref_float_to_half.restype = ctypes.c_uint16
        L.ref_set_threads.argtypes = [ctypes.c_int]
        L.ref_set_threads.restype = None
        _lib = L
    return _lib


def set_threads(n):
    """OpenMP threads of the C restatement (bench.py cpu_baseline: the host's cores)."""
    lib().ref_set_threads(int(n))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# --------------------------------------------------------------------------
# matching
# --------------------------------------------------------------------------
def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh,
              contract=False):
    """matching_kernels.cu:119-316 restated (oracle/matching_ref.c).  contract=True: the
    FMA-contracted model of nvcc's default --fmad=true (ref_iter_proj_fma)."""
    rays = _c(rays_img_with_grad, np.float32)
    pts = _c(pts_3d_norm, np.float32)
    pin = _c(p_init, np.float32)
    b, h, w, c = rays.shape
    n = pts.shape[1]
    p_new = np.zeros((b, n, 2), np.float32)
    conv = np.zeros((b, n), np.uint8)
    fn = lib().ref_iter_proj_fma if contract else lib().ref_iter_proj
    fn(_p(rays), _p(pts), _p(pin), _p(p_new), _p(conv), b, h, w, n, c, int(max_iter),
       float(lambda_init), float(cost_thresh))
    return p_new, conv.astype(bool)


def refine_matches(D11, D21, p1, radius, dilation_max):
    """matching_kernels.cu:25-116 restated; D11/D21 are float16 arrays."""
    d11 = _c(D11, np.float16).view(np.uint16)
    d21 = _c(D21, np.float16).view(np.uint16)
    p1 = _c(p1, np.int64)
    b, h, w, f = d11.shape
    n = d21.shape[1]
    out = np.zeros((b, n, 2), np.int64)
    lib().ref_refine_matches(_p(d11), _p(d21), _p(p1), _p(out), b, h, w, n, f, int(radius),
                             int(dilation_max))
    return out


def prep_for_iter_proj(X11, X21, idx_init=None):
    """matching.py:25-49 + image.py:5-38 (oracle/matching_ref.c ref_match_prep)."""
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    b, h, w, _ = X11.shape
    rwg = np.zeros((b, h, w, 9), np.float32)
    pts = np.zeros((b, h * w, 3), np.float32)
    p_init = np.zeros((b, h * w, 2), np.float32)
    idx = None if idx_init is None else _c(idx_init, np.int64)
    lib().ref_match_prep(_p(X11), _p(X21), _p(idx) if idx is not None else None, _p(rwg),
                         _p(pts), _p(p_init), b, h, w)
    return rwg, pts, p_init


def match_occlusion(X11, X21, p, conv, dist_thresh):
    """matching.py:67-76 → (p1 int64 [b,n,2], valid bool [b,n])."""
    X11 = _c(X11, np.float32)
    X21 = _c(X21, np.float32)
    p = _c(p, np.float32)
    conv = _c(conv, np.uint8)
    b, h, w, _ = X11.shape
    p1 = np.zeros((b, h * w, 2), np.int64)
    valid = np.zeros((b, h * w), np.uint8)
    lib().ref_match_occlusion(_p(X11), _p(X21), _p(p), _p(conv), _p(p1), _p(valid), b, h, w,
                              float(dist_thresh))
    return p1, valid.astype(bool)


def match(X11, X21, D11, D21, idx_init=None, cfg=None, contract=False, stages=False):
    """matching.match_iterative_proj (matching.py:52-90) restated on the CPU.  contract: the
    FMA-contracted iter_proj model; stages: also return the intermediate (p, converged)."""
    cfg = cfg or dict(max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6, dist_thresh=1e-1,
                      radius=3, dilation_max=5)
    b, h, w = X21.shape[:3]
    rwg, pts, p_init = prep_for_iter_proj(X11, X21, idx_init)
    p, conv = iter_proj(rwg, pts, p_init, cfg["max_iter"], cfg["lambda_init"],
                        cfg["convergence_thresh"], contract=contract)
    p1, valid = match_occlusion(X11, X21, p, conv, cfg["dist_thresh"])
    if cfg["radius"] > 0:
        p1 = refine_matches(D11.astype(np.float16), D21.reshape(b, h * w, -1).astype(np.float16),
                            p1, cfg["radius"], cfg["dilation_max"])
    idx = p1[..., 0] + w * p1[..., 1]
    if stages:
        return idx, valid[..., None], p, conv
    return idx, valid[..., None]


# --------------------------------------------------------------------------
# backend GN
# --------------------------------------------------------------------------
class _GnParams(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("sig0", ctypes.c_float), ("sig1", ctypes.c_float),
                ("C_thresh", ctypes.c_float), ("Q_thresh", ctypes.c_float),
                ("height", ctypes.c_int), ("width", ctypes.c_int),
                ("pixel_border", ctypes.c_int), ("z_eps", ctypes.c_float),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float)]


def gauss_newton(mode, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, *, sig0, sig1=1.0,
                 C_thresh, Q_thresh, max_iter, delta_thresh, K=None, height=0, width=0,
                 pixel_border=0, z_eps=0.0, want_first_system=False):
    """gn_kernels.cu gauss_newton_{rays,calib,points}_cuda restated.
    mode: 'rays' | 'calib' | 'points'.  Twc is updated in place (like the reference)."""
    prm = _GnParams()
    prm.mode = {"rays": 0, "calib": 1, "points": 2}[mode]
    prm.sig0, prm.sig1 = sig0, sig1
    prm.C_thresh, prm.Q_thresh = C_thresh, Q_thresh
    prm.height, prm.width, prm.pixel_border, prm.z_eps = height, width, pixel_border, z_eps
    if K is not None:
        K = np.asarray(K, np.float32)
        prm.fx, prm.fy, prm.cx, prm.cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    assert Twc.dtype == np.float32 and Twc.flags.c_contiguous
    Xs = _c(Xs, np.float32)
    Cs = _c(Cs, np.float32)
    ii = _c(ii, np.int64)
    jj = _c(jj, np.int64)
    idx = _c(idx_ii2jj, np.int64)
    vm = _c(valid_match, np.uint8)
    Q = _c(Q, np.float32)
    P, N = Xs.shape[:2]
    E = ii.shape[0]
    dx = np.zeros((max(P - 1, 0), 7), np.float32)
    H0 = np.zeros((E, 4, 7, 7), np.float64) if want_first_system else None
    g0 = np.zeros((E, 2, 7), np.float64) if want_first_system else None
    not_pd = ctypes.c_int(0)
    iters = lib().ref_gauss_newton(
        ctypes.byref(prm), _p(Twc), _p(Xs), _p(Cs), _p(ii), _p(jj), _p(idx), _p(vm), _p(Q), P, N,
        E, int(max_iter), float(delta_thresh), _p(dx), _p(H0) if H0 is not None else None,
        _p(g0) if g0 is not None else None, ctypes.byref(not_pd))
    out = dict(dx=dx, iters=iters, not_pd=bool(not_pd.value))
    if want_first_system:
        out["H"], out["g"] = H0, g0
    return out


def retr_sim3(xi, pose):
    xi = _c(xi, np.float32)
    pose = _c(pose, np.float32)
    out = np.zeros(8, np.float32)
    lib().ref_retr_sim3(_p(xi), _p(pose), _p(out))
    return out


def rel_sim3(Ti, Tj):
    Ti = _c(Ti, np.float32)
    Tj = _c(Tj, np.float32)
    out = np.zeros(8, np.float32)
    lib().ref_rel_sim3(_p(Ti), _p(Tj), _p(out))
    return out
