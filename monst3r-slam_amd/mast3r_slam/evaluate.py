"""mast3r_slam.evaluate (evaluate.py:24-45,110-141): TUM trajectory writers (+ ATE)."""
from monst3r_slam_amd.evaluate import (as_SE3, ate, ate_arrays, read_tum,  # noqa: F401
                                       save_full_traj, save_traj)
