"""mast3r_slam.nonlinear_optimizer (nonlinear_optimizer.py:5-33), restated."""
import math

import torch


def check_convergence(iter, rel_error_threshold, delta_norm_threshold, old_cost, new_cost,
                      delta, verbose=False):
    """Converged when |Δcost / old_cost| < rel_error_threshold or ‖delta‖ <
    delta_norm_threshold (old_cost = inf on the first iteration makes the ratio NaN: only
    the step-size test can fire there)."""
    rel_dec = math.fabs((old_cost - new_cost) / old_cost)
    delta_norm = torch.linalg.norm(delta)
    converged = rel_dec < rel_error_threshold or delta_norm < delta_norm_threshold
    if verbose:
        print(f"{iter=} | {new_cost=} {rel_dec=} {delta_norm=} | {converged=}")
    return converged


def huber(r, k=1.345):
    """IRLS Huber weight: 1 where |r| < k, else k / |r|."""
    a = torch.abs(r)
    return torch.where(a < k, torch.ones_like(r), k / a)
