"""mast3r_slam.global_opt2 (global_opt2.py:16-221): FactorGraph on the MI355X path."""
from monst3r_slam_amd.global_opt import FactorGraph, constrain_points_to_ray  # noqa: F401
