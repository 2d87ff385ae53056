"""mast3r_slam.lietorch_utils (lietorch_utils.py:6-14)."""
import torch

from monst3r_slam_amd.lie import SE3, Sim3


def as_SE3(X):
    """Drop the scale of a Sim3 (data [..., 8] → SE3 data [..., 7] as lietorch.SE3 keeps
    t, q); accepts Sim3 objects or raw data."""
    d = X.data if isinstance(X, Sim3) else X
    return SE3(torch.cat([d[..., :7], torch.ones_like(d[..., 7:8])], -1))
