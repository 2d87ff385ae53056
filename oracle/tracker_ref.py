"""ORACLE — test infrastructure only.

numpy restatement of the reference's frontend pose optimisation:
  FrameTracker2.solve                 tracker2.py:299-314
  FrameTracker2.opt_pose_ray_dist_sim3 tracker2.py:316-357
  FrameTracker2.opt_pose_calib_sim3    tracker2.py:359-409
  geometry.act_Sim3 / point_to_ray_dist / project_calib   geometry.py:17-104
  nonlinear_optimizer.check_convergence / huber            nonlinear_optimizer.py:5-33
lietorch (Sim3 act / inv / * / retr) is an external, unvendored dependency
(pyproject.toml:15, unpinned git URL, not installed here): its group operations are
restated from lietorch's published formulas as the reference itself restates them in
gn_kernels.cu:178-413 (oracle/gn_ref.c ref_retr_sim3 / ref_rel_sim3).  Parity with
lietorch itself is therefore UNPINNED (no reference test or fixture covers it).
All arithmetic in float32 like the reference's torch code, except the 7x7 Cholesky,
which torch runs in float32 too — here float64 (a tolerance, not a bit-exact, check).
"""
from __future__ import annotations

import math

import numpy as np

from . import oracle as _o


class CholeskyError(RuntimeError):
    pass


def _quat_rot(q):
    x, y, z, w = [float(v) for v in q]
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]],
                    np.float32)


def act(T, X):
    R = _quat_rot(T[3:7])
    return (np.float32(T[7]) * (X @ R.T) + T[:3].astype(np.float32)).astype(np.float32)


def mul(A, B):
    qa, qb = A[3:7].astype(np.float64), B[3:7].astype(np.float64)
    x1, y1, z1, w1 = qa
    x2, y2, z2, w2 = qb
    q = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                  w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    t = A[:3].astype(np.float64) + float(A[7]) * (_quat_rot(qa).astype(np.float64)
                                                  @ B[:3].astype(np.float64))
    return np.concatenate([t, q, [float(A[7]) * float(B[7])]]).astype(np.float32)


def skew(P):
    o = np.zeros_like(P[:, 0])
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    return np.stack([o, -z, y, z, o, -x, -y, x, o], -1).reshape(-1, 3, 3)


def act_jac(T, X):
    """geometry.act_Sim3(jacobian=True): P, [I, -[P]x, P]."""
    P = act(T, X)
    n = P.shape[0]
    J = np.concatenate([np.broadcast_to(np.eye(3, dtype=np.float32), (n, 3, 3)), -skew(P),
                        P[:, :, None]], axis=-1)
    return P, J.astype(np.float32)


def point_to_ray_dist(X, jacobian=False):
    d = np.sqrt((X * X).sum(-1, keepdims=True)).astype(np.float32)
    d_inv = (np.float32(1.0) / d).astype(np.float32)
    r = d_inv * X
    rd = np.concatenate([r, d], -1)
    if not jacobian:
        return rd
    d_inv_2 = d_inv ** 2
    I = np.eye(3, dtype=np.float32)
    dr_dX = d_inv[..., None] * (I - d_inv_2[..., None] * (X[:, :, None] * X[:, None, :]))
    drd = np.concatenate([dr_dX, r[:, None, :]], axis=1)
    return rd, drd.astype(np.float32)


def project_calib(P, K, img_size, border, z_eps):
    p = P @ K.T
    p = p / p[:, 2:3]
    u, v = p[:, 0:1], p[:, 1:2]
    x, y, z = P[:, 0:1], P[:, 1:2], P[:, 2:3]
    valid = ((u > border) & (u < img_size[1] - 1 - border) & (v > border)
             & (v < img_size[0] - 1 - border) & (z > z_eps))
    with np.errstate(all="ignore"):
        logz = np.where(z > z_eps, np.log(np.where(z > 0, z, 1)), 0).astype(np.float32)
        z_inv = (np.float32(1.0) / z[:, 0]).astype(np.float32)
    fx, fy = K[0, 0], K[1, 1]
    J = np.zeros((P.shape[0], 3, 3), np.float32)
    J[:, 0, 0] = fx
    J[:, 1, 1] = fy
    J[:, 0, 2] = -fx * x[:, 0] * z_inv
    J[:, 1, 2] = -fy * y[:, 0] * z_inv
    J *= z_inv[:, None, None]
    J[:, 2, 2] = z_inv
    return np.concatenate([p[:, :2], logz], -1).astype(np.float32), J, valid


def huber(r, k):
    a = np.abs(r)
    with np.errstate(divide="ignore"):
        return np.where(a < k, np.float32(1), np.float32(k) / a).astype(np.float32)


def solve(sqrt_info, r, J, huber_k):
    whitened = sqrt_info * r
    robust = sqrt_info * np.sqrt(huber(whitened, huber_k))
    A = (robust[..., None] * J).reshape(-1, 7).astype(np.float32)
    b = (robust * r).reshape(-1, 1).astype(np.float32)
    H = (A.T.astype(np.float64) @ A.astype(np.float64))
    g = -(A.T.astype(np.float64) @ b.astype(np.float64))
    cost = 0.5 * float((b.astype(np.float64) ** 2).sum())
    try:
        L = np.linalg.cholesky(H)
    except np.linalg.LinAlgError as e:
        raise CholeskyError(str(e))
    tau = np.linalg.solve(L.T, np.linalg.solve(L, g)).reshape(-1).astype(np.float32)
    return tau, cost


def converged(old_cost, new_cost, tau, rel_error, delta_norm):
    with np.errstate(invalid="ignore"):
        rel_dec = abs((old_cost - new_cost) / old_cost) if old_cost != math.inf else math.nan
    return (rel_dec < rel_error) or (float(np.linalg.norm(tau)) < delta_norm)


def opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg):
    vq = valid.astype(np.float32)[:, None] * np.sqrt(Qk.astype(np.float32))[:, None]
    si = np.concatenate([np.float32(1 / cfg["sigma_ray"]) * vq.repeat(3, 1),
                         np.float32(1 / cfg["sigma_dist"]) * vq], 1)
    T = _o.rel_sim3(T_WCk, T_WCf)
    rd_k = point_to_ray_dist(Xk)
    old_cost = math.inf
    it = 0
    for it in range(cfg["max_iters"]):
        P, Ja = act_jac(T, Xf)
        rd, drd = point_to_ray_dist(P, jacobian=True)
        r = rd_k - rd
        J = -np.einsum("nij,njk->nik", drd, Ja)
        tau, new_cost = solve(si, r, J, cfg["huber"])
        T = _o.retr_sim3(tau, T)
        if converged(old_cost, new_cost, tau, cfg["rel_error"], cfg["delta_norm"]):
            break
        old_cost = new_cost
    return mul(T_WCk, T), T, it + 1


def opt_pose_calib_sim3(Xf, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size, cfg):
    vq = valid.astype(np.float32)[:, None] * np.sqrt(Qk.astype(np.float32))[:, None]
    si = np.concatenate([np.float32(1 / cfg["sigma_pixel"]) * vq.repeat(2, 1),
                         np.float32(1 / cfg["sigma_depth"]) * vq], 1)
    T = _o.rel_sim3(T_WCk, T_WCf)
    old_cost = math.inf
    it = 0
    for it in range(cfg["max_iters"]):
        P, Ja = act_jac(T, Xf)
        pz, dpz, vproj = project_calib(P, K, img_size, cfg["pixel_border"], cfg["depth_eps"])
        si2 = (vproj & valid_meas_k[:, None]).astype(np.float32) * si
        r = meas_k - pz
        J = -np.einsum("nij,njk->nik", dpz, Ja)
        tau, new_cost = solve(si2, r, J, cfg["huber"])
        T = _o.retr_sim3(tau, T)
        if converged(old_cost, new_cost, tau, cfg["rel_error"], cfg["delta_norm"]):
            break
        old_cost = new_cost
    return mul(T_WCk, T), T, it + 1
