"""Configuration: same YAML keys and `inherit:` merge as mast3r_slam/config.py:7-54.

`default_config()` returns the values of the reference's config/base.yaml:15-57 for the
keys the hot path reads (matching, tracking, local_opt)."""
from __future__ import annotations

import copy
import re

import yaml

_BASE = {
    "use_calib": False,
    "use_dynamic_mask": False,
    "dataset": {"subsample": 1, "img_downsample": 1, "center_principle_point": True},
    "matching": {"max_iter": 10, "lambda_init": 1e-8, "convergence_thresh": 1e-6,
                 "dist_thresh": 1e-1, "radius": 3, "dilation_max": 5},
    "tracking": {"min_match_frac": 0.05, "max_iters": 50, "C_conf": 0.0, "Q_conf": 1.5,
                 "rel_error": 1e-3, "delta_norm": 1e-3, "huber": 1.345,
                 "match_frac_thresh": 0.333, "sigma_ray": 0.003, "sigma_dist": 1e1,
                 "sigma_pixel": 1.0, "sigma_depth": 1e1, "sigma_point": 0.05,
                 "pixel_border": -10, "depth_eps": 1e-6, "filtering_mode": "weighted_pointmap",
                 "filtering_score": "median"},
    "local_opt": {"pin": 1, "window_size": 1e6, "C_conf": 0.0, "Q_conf": 1.5,
                  "min_match_frac": 0.1, "pixel_border": -10, "depth_eps": 1e-6,
                  "max_iters": 10, "sigma_ray": 0.003, "sigma_dist": 1e1, "sigma_pixel": 1.0,
                  "sigma_depth": 1e1, "sigma_point": 0.05, "delta_norm": 1e-8,
                  "use_cuda": True},
    "retrieval": {"k": 3, "min_thresh": 5e-3},
    "reloc": {"min_match_frac": 0.3, "strict": True},
}

config: dict = copy.deepcopy(_BASE)


def default_config() -> dict:
    return copy.deepcopy(_BASE)


def _loader():
    loader = yaml.SafeLoader
    loader.add_implicit_resolver(
        "tag:yaml.org,2002:float",
        re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                    |\.[0-9_]+(?:[eE][-+][0-9]+)?
                    |[-+]?\.(?:inf|Inf|INF)|\.(?:nan|NaN|NAN))$""", re.X),
        list("-+0123456789."))
    return loader


def _merge(a: dict, b: dict) -> dict:
    for k, v in b.items():
        if isinstance(v, dict):
            a[k] = _merge(a.get(k, {}) if isinstance(a.get(k), dict) else {}, v)
        else:
            a[k] = v
    return a


def load_config(path: str, _is_parent: bool = False) -> dict:
    with open(path) as f:
        cfg = yaml.load(f, Loader=_loader())
    parent = load_config(cfg["inherit"], True) if cfg.get("inherit") else {}
    cfg = _merge(parent, cfg)
    if not _is_parent:
        config.clear()
        config.update(_merge(default_config(), cfg))
    return cfg
