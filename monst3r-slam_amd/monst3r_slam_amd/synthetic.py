"""Seeded synthetic inputs for tests and bench (no datasets or checkpoints offline).

Scene model: a textured analytic depth surface seen by a pinhole
camera (fx = fy = 400, cx = w/2, cy = h/2), a smooth Sim3 trajectory, pointmaps
X = backproject(pixel, z) (+ small noise), confidences C = 1 + exp(N(1, .5)),
descriptors D = normalize(R f(x, y)) (fixed random projection of a smooth texture
field evaluated at the surface point), Q = exp(N(1, .5)).
"""
from __future__ import annotations

import math

import numpy as np


def intrinsics(h: int, w: int) -> np.ndarray:
    return np.array([[400.0, 0.0, w / 2.0], [0.0, 400.0, h / 2.0], [0.0, 0.0, 1.0]], np.float32)


def quat_from_axis_angle(axis, angle):
    axis = np.asarray(axis, np.float64)
    axis = axis / (np.linalg.norm(axis) + 1e-300)
    s = math.sin(angle / 2.0)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, math.cos(angle / 2.0)], np.float64)


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def sim3_act(T, X):
    """T = [t(3), q xyzw(4), s] acting on points [..., 3] (s R X + t)."""
    R = quat_to_rot(np.asarray(T[3:7], np.float64))
    return (T[7] * (X.astype(np.float64) @ R.T) + np.asarray(T[:3], np.float64)).astype(np.float32)


def sim3_inv(T):
    R = quat_to_rot(np.asarray(T[3:7], np.float64))
    s = float(T[7])
    t = -(R.T @ np.asarray(T[:3], np.float64)) / s
    q = np.array([-T[3], -T[4], -T[5], T[6]], np.float64)
    return np.concatenate([t, q, [1.0 / s]]).astype(np.float32)


def sim3_mul(A, B):
    """A * B."""
    qa, qb = np.asarray(A[3:7], np.float64), np.asarray(B[3:7], np.float64)
    x1, y1, z1, w1 = qa
    x2, y2, z2, w2 = qb
    q = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                  w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    t = np.asarray(A[:3], np.float64) + float(A[7]) * (quat_to_rot(qa) @ np.asarray(B[:3],
                                                                                   np.float64))
    return np.concatenate([t, q, [float(A[7]) * float(B[7])]]).astype(np.float32)


def depth_surface(h, w, seed=0, phase=0.0):
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64),
                         indexing="ij")
    z = 2.5 + 0.4 * np.sin(xx / 37.0 + phase + rng.uniform(0, 1)) * np.cos(yy / 29.0)
    z += 0.25 * np.sin((xx + yy) / 61.0 + rng.uniform(0, 6))
    return z.astype(np.float32)


def backproject(z, K):
    h, w = z.shape
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32),
                         indexing="ij")
    X = np.stack([(xx - K[0, 2]) / K[0, 0] * z, (yy - K[1, 2]) / K[1, 1] * z, z], axis=-1)
    return X.astype(np.float32)


def texture_field(P, dim=24, seed=7):
    """Smooth random feature field of 3-D points → unit 24-d descriptors."""
    rng = np.random.default_rng(seed)
    freqs = rng.normal(0, 3.0, size=(dim * 2, 3)).astype(np.float32)
    phases = rng.uniform(0, 2 * np.pi, size=(dim * 2,)).astype(np.float32)
    feats = np.sin(P @ freqs.T + phases)
    R = rng.normal(0, 1, size=(dim * 2, dim)).astype(np.float32)
    D = feats @ R
    return (D / np.linalg.norm(D, axis=-1, keepdims=True)).astype(np.float32)


def pair(h=384, w=512, seed=0, shift_px=(1.5, -0.75), noise=1e-3):
    """A matching test pair: X11 (view-1 pointmap), X21 (view-2 pixels' points in frame 1,
    from a sub-pixel image-plane shift of the same surface), descriptors D11/D21."""
    rng = np.random.default_rng(seed)
    K = intrinsics(h, w)
    z = depth_surface(h, w, seed)
    X11 = backproject(z, K)
    # view 2 pixel (x, y) sees the surface point at view-1 pixel (x + sx, y + sy)
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32),
                         indexing="ij")
    xs = np.clip(xx + shift_px[0], 0, w - 1)
    ys = np.clip(yy + shift_px[1], 0, h - 1)
    x0 = np.floor(xs).astype(np.int64)
    y0 = np.floor(ys).astype(np.int64)
    x1 = np.minimum(x0 + 1, w - 1)
    y1 = np.minimum(y0 + 1, h - 1)
    fx = (xs - x0)[..., None]
    fy = (ys - y0)[..., None]
    X21 = ((1 - fx) * (1 - fy) * X11[y0, x0] + fx * (1 - fy) * X11[y0, x1]
           + (1 - fx) * fy * X11[y1, x0] + fx * fy * X11[y1, x1]).astype(np.float32)
    X21 = X21 * (1.0 + noise * rng.normal(size=X21.shape[:-1] + (1,))).astype(np.float32)
    D11 = texture_field(X11)
    D21 = texture_field(X21)
    return X11, X21, D11, D21


def pointmap_pair_batch(b, h, w, seed=0):
    Xs, Ys, Ds, Es = [], [], [], []
    for i in range(b):
        X11, X21, D11, D21 = pair(h, w, seed + i, shift_px=(1.0 + 0.5 * i, -0.5 + 0.25 * i))
        Xs.append(X11)
        Ys.append(X21)
        Ds.append(D11)
        Es.append(D21)
    return np.stack(Xs), np.stack(Ys), np.stack(Ds), np.stack(Es)


def keyframe_graph(P=5, h=48, w=64, seed=0, noise=1e-3, perturb=0.01, pairs=None,
                   two_way=False):
    """Backend GN test problem: P keyframes observing the same world points Xw (the view-0
    surface) under a smooth Sim3 trajectory; keyframe k's pointmap is T_k^-1 Xw (+ noise),
    so the true correspondence of every edge is the identity index (90 % marked valid).
    Edges (i, i+1), (i, i+2) — or, with `pairs=n`, the first n pairs (i, i+g) by gap
    g = 1, 2, ... (the covisibility bands a keyframe graph holds), each also as (j, i) when
    `two_way` (FactorGraph.add_factors' two-way packing).  Initial poses 1..P-1 perturbed
    by ~`perturb`."""
    rng = np.random.default_rng(seed)
    K = intrinsics(h, w)
    N = h * w
    T_gt = []
    for k in range(P):
        q = quat_from_axis_angle([0.3, 1.0, 0.2], 0.03 * k)
        t = np.array([0.05 * k, -0.02 * k, 0.01 * k])
        T_gt.append(np.concatenate([t, q, [1.0 + 0.01 * k]]).astype(np.float32))
    Xw = backproject(depth_surface(h, w, seed), K).reshape(-1, 3)
    Xs = np.stack([sim3_act(sim3_inv(T), Xw) for T in T_gt]).astype(np.float32)
    Xs = Xs * (1.0 + noise * rng.normal(size=Xs.shape[:-1] + (1,))).astype(np.float32)
    if pairs is None:
        edges = [(i, i + 1) for i in range(P - 1)] + [(i, i + 2) for i in range(P - 2)]
    else:
        edges = [(i, i + g) for g in range(1, P) for i in range(P - g)][:pairs]
    if two_way:
        edges = edges + [(j, i) for i, j in edges]
    ii = np.array([e[0] for e in edges], np.int64)
    jj = np.array([e[1] for e in edges], np.int64)
    E = len(edges)
    idx = np.tile(np.arange(N, dtype=np.int64)[None], (E, 1))
    valid = rng.uniform(size=(E, N, 1)) < 0.9
    Q = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(E, N, 1)))).astype(np.float32)
    Cs = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(P, N, 1)))).astype(np.float32)
    Twc_gt = np.stack(T_gt).astype(np.float32)
    Twc = Twc_gt.copy()
    for k in range(1, P):
        d = rng.normal(0, perturb, 7)
        q = quat_from_axis_angle(d[3:6], np.linalg.norm(d[3:6]))
        Twc[k] = sim3_mul(np.concatenate([d[:3], q, [math.exp(d[6])]]).astype(np.float32),
                          Twc[k])
    return dict(Twc_gt=Twc_gt, Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx=idx, valid=valid, Q=Q,
                K=K, h=h, w=w)


def tracking_problem(h=384, w=512, seed=0, noise=1e-3, valid_frac=0.95):
    """Frontend tracking test: keyframe pointmap Xk (camera k), frame points
    Xf = T_CkCf_gt^-1 Xk (+ noise) with identity correspondence, Qk, valid, calibrated
    measurements meas_k = (u, v, log z_k).  T_WCf starts at T_WCk (identity relative)."""
    rng = np.random.default_rng(seed)
    K = intrinsics(h, w)
    Xk = backproject(depth_surface(h, w, seed), K).reshape(-1, 3)
    q = quat_from_axis_angle([0.2, 1.0, -0.3], 0.02)
    T_gt = np.concatenate([[0.03, -0.01, 0.02], q, [1.01]]).astype(np.float32)
    Xf = sim3_act(sim3_inv(T_gt), Xk)
    Xf = (Xf * (1.0 + noise * rng.normal(size=(Xf.shape[0], 1)))).astype(np.float32)
    Qk = (1.0 + np.exp(rng.normal(1.0, 0.5, size=Xk.shape[0]))).astype(np.float32)
    valid = rng.uniform(size=Xk.shape[0]) < valid_frac
    qk = quat_from_axis_angle([1.0, 0.0, 0.5], 0.1)
    T_WCk = np.concatenate([[0.5, 0.1, -0.2], qk, [1.2]]).astype(np.float32)
    T_WCf = T_WCk.copy()
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32),
                         indexing="ij")
    meas_k = np.stack([xx.reshape(-1), yy.reshape(-1), np.log(Xk[:, 2])], -1).astype(np.float32)
    valid_meas = Xk[:, 2] > 1e-6
    return dict(Xf=Xf, Xk=Xk, Qk=Qk, valid=valid, T_WCk=T_WCk, T_WCf=T_WCf, T_gt=T_gt, K=K,
                meas_k=meas_k, valid_meas=valid_meas, h=h, w=w)


def tracking_sequence(n=8, h=96, w=128, seed=0, noise=1e-3):
    """A sequence with ground truth for the headless harness: one keyframe surface X_key
    (world = keyframe camera) and n frames with GT Sim3 poses T_t (frame -> world).  Frame t's
    pair outputs are what a perfect network would regress: Xji = T_t^-1 X_key on the keyframe
    pixels, Xii = T_t^-1 of the surface seen with a sub-pixel image shift, descriptors from the
    world points.  Returns (X_key [N,3], frames [dict X, C, D16, Q numpy], T_gt [n, 8])."""
    rng = np.random.default_rng(seed)
    K = intrinsics(h, w)
    X_key = backproject(depth_surface(h, w, seed), K)
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32),
                         indexing="ij")
    frames, T_gt = [], []
    for t in range(n):
        q = quat_from_axis_angle([0.3, 1.0, -0.2], 0.004 * t)
        T = np.concatenate([[0.004 * t, -0.002 * t, 0.003 * t], q, [1.0 + 0.002 * t]])
        T = T.astype(np.float32)
        sx, sy = 0.5 + 0.2 * np.sin(t), -0.3 + 0.2 * np.cos(t)
        xs, ys = np.clip(xx + sx, 0, w - 1), np.clip(yy + sy, 0, h - 1)
        x0, y0 = np.floor(xs).astype(np.int64), np.floor(ys).astype(np.int64)
        x1, y1 = np.minimum(x0 + 1, w - 1), np.minimum(y0 + 1, h - 1)
        fx, fy = (xs - x0)[..., None], (ys - y0)[..., None]
        Xw = ((1 - fx) * (1 - fy) * X_key[y0, x0] + fx * (1 - fy) * X_key[y0, x1]
              + (1 - fx) * fy * X_key[y1, x0] + fx * fy * X_key[y1, x1]).astype(np.float32)
        Tinv = sim3_inv(T)
        Xii = sim3_act(Tinv, Xw.reshape(-1, 3)).reshape(h, w, 3)
        Xii = Xii * (1.0 + noise * rng.normal(size=(h, w, 1)))
        Xji = sim3_act(Tinv, X_key.reshape(-1, 3)).reshape(h, w, 3)
        D = np.stack([texture_field(Xw), texture_field(X_key)]).astype(np.float16)
        C = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, h, w)))).astype(np.float32)
        Q = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, h, w)))).astype(np.float32)
        frames.append(dict(X=np.stack([Xii, Xji]).astype(np.float32), C=C, D16=D, Q=Q))
        T_gt.append(T)
    return X_key.reshape(-1, 3).astype(np.float32), frames, np.stack(T_gt)
