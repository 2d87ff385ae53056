"""mast3r_slam.matching (matching.py:8-90) on the fused HIP kernels."""
from monst3r_slam_amd.matching import (lin_to_pixel, match, match_iterative_proj,  # noqa: F401
                                       pixel_to_lin, prep_for_iter_proj)
