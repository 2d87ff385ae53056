"""ctypes binding of the C-ABI library libmonst3r_slam_amd.so (include/monst3r_slam_amd.h).

The HIP library is the product path: if it is missing this module raises; there is no
CPU or PyTorch fallback.  torch is imported first so that torch's libamdhip64.so.7 is the
one HIP runtime in the process (same SONAME; the loader reuses it for this library).
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("M3S_LIB_PATH") or os.path.join(_HERE, "libmonst3r_slam_amd.so")  # A/B builds
HEADER = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "monst3r_slam_amd.h"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/monst3r_slam_amd.h
SIGNATURES = {
    "m3s_status_string": (ctypes.c_char_p, [_I]),
    "m3s_version": (_I, []),
    "m3s_device_count": (_I, []),
    "m3s_timeline_set": (_I, [_P, _I]),
    "m3s_timeline_count": (_I, []),
    "m3s_timeline_meta": (_I, [_P, _P, _P, _I]),
    "m3s_iter_proj": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _F, _F, _P]),
    "m3s_iter_proj_fma": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _F, _F, _P]),
    "m3s_refine_matches": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I, _I, _P]),
    "m3s_match_prep": (_I, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P]),
    "m3s_match_occlusion": (_I, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _F, _P]),
    "m3s_pixel_to_lin": (_I, [_P, _P, _I64, _I64, _I64, _P]),
    "m3s_gn_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "m3s_gauss_newton_rays": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _F, _F, _F,
                                   _F, _I, _F, _P, _P, _P, _P]),
    "m3s_gauss_newton_calib": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I, _I,
                                    _I, _F, _F, _F, _F, _F, _I, _F, _P, _P, _P, _P]),
    "m3s_gauss_newton_points": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _F, _F,
                                     _F, _I, _F, _P, _P, _P, _P]),
    "m3s_gn_force_global_solve": (_I, [_I]),
    "m3s_gn_sharded_workspace_bytes": (_SZ, [_I64, _I64, _I64, _I64]),
    "m3s_gn_sharded_begin": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P, _P, _P]),
    "m3s_gn_rays_edge_pass": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _F,
                                   _F, _F, _P, _P, _P]),
    "m3s_gn_calib_edge_pass": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I,
                                    _I, _I, _F, _F, _F, _F, _F, _P, _P, _P]),
    "m3s_gn_solve_step": (_I, [_P, _P, _I64, _I64, _I64, _I64, _F, _P, _P, _P]),
    "m3s_gn_sharded_status": (_I, [_P, _I64, _P, _P, _P]),
    "m3s_track_workspace_bytes": (_SZ, [_I64]),
    "m3s_track_rays": (_I, [_P, _P, _P, _P, _P, _P, _I64, _F, _F, _F, _I, _F, _F, _P, _P, _P, _P,
                            _P]),
    "m3s_track_calib": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _F, _F, _F, _F, _F,
                             _I, _F, _F, _P, _P, _P, _P, _P]),
    "m3s_glue_workspace_bytes": (_SZ, [_I64]),
    "m3s_track_glue_pre": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _F, _F, _P, _P, _P, _P, _P]),
    "m3s_track_glue_post": (_I, [_P, _P, _P, _P, _P, _P, _I64, _F, _F, _P, _P, _P, _P, _P, _P,
                                 _P]),
    "m3s_vit_gemm": (_I, [_P, _P]),
    "m3s_vit_layernorm": (_I, [_P, _I, _P, _P, _P, _I, _I64, _I64, _F, _I64, _I64, _I64, _I64,
                               _I64, _I, _P]),
    "m3s_vit_layernorm_dual": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I64, _I64, _F, _I64, _I64, _I64,
                                    _I64, _I64, _P]),
    "m3s_vit_rope": (_I, [_P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "m3s_vit_attention": (_I, [_P, _I64, _I64, _P, _P, _I64, _I64, _P, _P, _I64, _P, _I64, _I64,
                               _I, _I64, _I64, _I64, _I64, _F, _P, _I64, _I, _P]),
    "m3s_vit_rope_table": (_I, [_P, _I64, _F, _P, _P]),
    "m3s_vit_patchify": (_I, [_P, _P, _I64, _I64, _I64, _P]),
    "m3s_copy_rows": (_I, [_P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64,
                           _I64, _I64, _P]),
    "m3s_vit_upsample2x": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "m3s_vit_upsample2x_e4m3": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _F, _P]),
    "m3s_vit_dpt_out": (_I, [_P, _P, _P, _P, _P, _I64, _F, _I64, _I64, _I64, _I64, _P]),
    "m3s_vit_local_features": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _P]),
    "m3s_ego_flow": (_I, [_P, _P, _I64, _I64, _P, _P]),
    "m3s_flow_error_mask": (_I, [_P, _P, _I64, _F, _P, _P, _P]),
    "m3s_apply_dynamic_mask": (_I, [_P, _P, _P, _P, _I, _I64, _I64, _I64, _F, _I, _P]),
    "m3s_retr_affine": (_I, [_P, _I, _I64, _P, _P, _P, _P, _I64, _I64, _I64, _P, _P]),
    "m3s_retr_rownorm": (_I, [_P, _I64, _I64, _I, _P, _P]),
    "m3s_topk_select": (_I, [_P, _I, _I64, _I64, _I, _P, _P, _P]),
    "m3s_retr_quantize_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "m3s_retr_quantize": (_I, [_P, _P, _I64, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P]),
    "m3s_asmk_aggregate": (_I, [_P, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _P, _P, _P]),
    "m3s_ivf_search": (_I, [_P, _P, _P, _I64, _P, _P, _P, _I64, _I64, _F, _F, _P, _P, _P]),
    "m3s_seq_gather": (_I, [_P, _I64, _P, _I, _I, _P, _P]),
    "m3s_seq_pair_outputs": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I64, _P, _P, _P, _P,
                                  _P]),
    "m3s_seq_advance": (_I, [_P, _P, _P, _P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                             _P, _P, _P, _I, _P]),
}


class GemmDesc(ctypes.Structure):
    """m3s_gemm_desc (include/monst3r_slam_amd.h)."""
    _fields_ = [("A", _P), ("lda", _I64), ("strideA", _I64),
                ("B", _P), ("ldb", _I64), ("strideB", _I64),
                ("C", _P), ("ldc", _I64), ("strideC", _I64),
                ("bias", _P), ("strideBias", _I64),
                ("R", _P), ("ldr", _I64), ("strideR", _I64),
                ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("flags", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("Hin", ctypes.c_int32), ("Win", ctypes.c_int32), ("Cin", ctypes.c_int32),
                ("Hout", ctypes.c_int32), ("Wout", ctypes.c_int32), ("stride", ctypes.c_int32),
                ("ct_s", ctypes.c_int32), ("ct_cout", ctypes.c_int32), ("ct_gw", ctypes.c_int32),
                ("workspace", _P), ("workspace_bytes", _I64), ("split_k", ctypes.c_int32),
                ("rope_table", _P), ("rope_cols", ctypes.c_int32),
                ("rope_tokens", ctypes.c_int32), ("weight_mod", ctypes.c_int32),
                ("dpt_w4", _P), ("dpt_b4", _P), ("dpt_pts", _P), ("dpt_conf", _P),
                ("dpt_conf_min", ctypes.c_float), ("col_scale", _P),
                ("stride_col_scale", _I64), ("C2", _P), ("stats", _P),
                ("stats_groups", ctypes.c_int32), ("a_batch_xor", ctypes.c_int32),
                ("ln_c1", _P), ("ln_eps", ctypes.c_float),
                ("tile_counters", _P), ("tile_counters_len", ctypes.c_int32),
                ("tile_hint", ctypes.c_int32),
                ("ln_c3", _P), ("ln_shift", _P), ("ln_qscale", _P)]


(EPI_BIAS, EPI_GELU, EPI_RELU, EPI_RES_F32, EPI_RES_BF16, EPI_OUT_F32, PRO_RELU, EPI_CONVT,
 EPI_ROPE, EPI_DPT_OUT, IN_FP8, EPI_OUT_FP8, EPI_LN_STATS, EPI_LN_FOLD) = (
    1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192)

_lib = None


def load():
    """Load (once) and return the native library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"monst3r_slam_amd: native HIP library not found at {LIB_PATH}; build it with "
                "`make -C monst3r-slam_amd/csrc` or `python -c 'import __graft_entry__ as g; "
                "g.build()'` (there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def status_string(status: int) -> str:
    return load().m3s_status_string(int(status)).decode()


def check(status: int, what: str):
    if status != 0:
        raise RuntimeError(f"{what}: {status_string(status)} (status {status})")


def ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors, names=()):
    for i, t in enumerate(tensors):
        if t is None:
            continue
        if not t.is_cuda:
            nm = names[i] if i < len(names) else f"arg{i}"
            raise RuntimeError(f"{nm} must be a GPU (HIP) tensor: the MI355X path has no CPU "
                               "fallback")


def require_contiguous(**tensors):
    # reference: CHECK_CONTIGUOUS → TORCH_CHECK(x.is_contiguous(), #x " must be contiguous")
    for name, t in tensors.items():
        if t is not None and not t.is_contiguous():
            raise RuntimeError(f"{name} must be contiguous")
