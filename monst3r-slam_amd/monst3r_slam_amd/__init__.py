"""MI355X-native host side of the MonST3R/MASt3R-SLAM per-frame hot path.

Mirrors the reference's operator API (mast3r_slam.matching, mast3r_slam.monst3r_utils,
tracker2 / global_opt2 solvers) on top of the HIP kernels in libmonst3r_slam_amd.so
(C ABI: include/monst3r_slam_amd.h).  No CPU fallback: every op requires the library.
"""
from .config import config, default_config, load_config  # noqa: F401

__version__ = "0.1.0"
