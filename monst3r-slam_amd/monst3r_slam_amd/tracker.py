"""Frontend pose optimisation — mirror of FrameTracker2.opt_pose_ray_dist_sim3 /
opt_pose_calib_sim3 (tracker2.py:316-409) on the fused HIP tracker kernels
(m3s_track_rays / m3s_track_calib).  Poses are lietorch Sim3 data tensors [8]
(t xyz, q xyzw, s).  Returns (T_WCf, T_CkCf, info) with info = [iters, chol_failed,
converged, recovered]; a failed Cholesky raises CholeskyError like torch.linalg.cholesky does
(tracker2.py:234-236 catches it and reports the frame lost)."""
from __future__ import annotations

import torch

from . import _lib
from .config import config as _config


class CholeskyError(RuntimeError):
    pass


def _ws(n, dev):
    return torch.empty((_lib.load().m3s_track_workspace_bytes(n),), dtype=torch.uint8,
                       device=dev)


def _prep(t, dtype=torch.float32):
    return t.to(dtype).contiguous()


def opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg=None, check=True):
    cfg = cfg or _config["tracking"]
    dev = Xf.device
    _lib.require_cuda(Xf, Xk, T_WCf, T_WCk, Qk, valid,
                      names=("Xf", "Xk", "T_WCf", "T_WCk", "Qk", "valid"))
    n = Xf.shape[0]
    Xf, Xk = _prep(Xf.reshape(n, 3)), _prep(Xk.reshape(n, 3))
    Qk = _prep(Qk.reshape(n))
    valid = valid.reshape(n).to(torch.uint8).contiguous()
    T_WCf, T_WCk = _prep(T_WCf.reshape(8)), _prep(T_WCk.reshape(8))
    out_f = torch.empty(8, dtype=torch.float32, device=dev)
    out_rel = torch.empty(8, dtype=torch.float32, device=dev)
    info = torch.empty(4, dtype=torch.int32, device=dev)  # track_finish writes all 4
    ws = _ws(n, dev)
    st = _lib.load().m3s_track_rays(
        _lib.ptr(T_WCk), _lib.ptr(T_WCf), _lib.ptr(Xf), _lib.ptr(Xk), _lib.ptr(Qk),
        _lib.ptr(valid), n, float(cfg["sigma_ray"]), float(cfg["sigma_dist"]),
        float(cfg["huber"]), int(cfg["max_iters"]), float(cfg["rel_error"]),
        float(cfg["delta_norm"]), _lib.ptr(out_f), _lib.ptr(out_rel), _lib.ptr(info),
        _lib.ptr(ws), _lib.stream(dev))
    _lib.check(st, "track_rays")
    if check and int(info[1].item()):
        raise CholeskyError("tracker: Cholesky failed (H not positive definite)")
    return out_f, out_rel, info


def opt_pose_calib_sim3(Xf, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size,
                        cfg=None, check=True):
    cfg = cfg or _config["tracking"]
    dev = Xf.device
    _lib.require_cuda(Xf, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K,
                      names=("Xf", "T_WCf", "T_WCk", "Qk", "valid", "meas_k", "valid_meas_k",
                             "K"))
    n = Xf.shape[0]
    Xf = _prep(Xf.reshape(n, 3))
    Qk = _prep(Qk.reshape(n))
    valid = valid.reshape(n).to(torch.uint8).contiguous()
    meas_k = _prep(meas_k.reshape(n, 3))
    valid_meas_k = valid_meas_k.reshape(n).to(torch.uint8).contiguous()
    K = _prep(K.reshape(3, 3))
    T_WCf, T_WCk = _prep(T_WCf.reshape(8)), _prep(T_WCk.reshape(8))
    out_f = torch.empty(8, dtype=torch.float32, device=dev)
    out_rel = torch.empty(8, dtype=torch.float32, device=dev)
    info = torch.empty(4, dtype=torch.int32, device=dev)  # track_finish writes all 4
    ws = _ws(n, dev)
    h, w = int(img_size[0]), int(img_size[1])
    st = _lib.load().m3s_track_calib(
        _lib.ptr(T_WCk), _lib.ptr(T_WCf), _lib.ptr(Xf), _lib.ptr(Qk), _lib.ptr(valid),
        _lib.ptr(meas_k), _lib.ptr(valid_meas_k), _lib.ptr(K), n, h, w,
        float(cfg["sigma_pixel"]), float(cfg["sigma_depth"]), float(cfg["huber"]),
        float(cfg["pixel_border"]), float(cfg["depth_eps"]), int(cfg["max_iters"]),
        float(cfg["rel_error"]), float(cfg["delta_norm"]), _lib.ptr(out_f), _lib.ptr(out_rel),
        _lib.ptr(info), _lib.ptr(ws), _lib.stream(dev))
    _lib.check(st, "track_calib")
    if check and int(info[1].item()):
        raise CholeskyError("tracker: Cholesky failed (H not positive definite)")
    return out_f, out_rel, info
