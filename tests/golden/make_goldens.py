"""Generate the matching-prep golden fixtures FROM THE REFERENCE's own Python code.

Container-only (needs /root/reference; never run on the GPU box).  Imports
/root/reference/MASt3R-SLAM/mast3r_slam/matching.py (+ image.py, config.py) on the CPU.
Its native module `mast3r_slam_backends` is CUDA-only and absent, so a module object whose
iter_proj / refine_matches return pre-drawn arrays is placed in sys.modules: the golden
then pins the reference's Python glue around the kernels (prep_for_iter_proj :25-49,
img_gradient, the occlusion test :67-76 and pixel_to_lin :13-15,88) on fixed inputs.

Writes tests/golden/matching_prep.npz.  Run:  python tests/golden/make_goldens.py
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/MASt3R-SLAM"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "matching_prep.npz")


def main():
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    b, h, w = 2, 24, 32
    n = h * w
    # smooth positive-depth pointmaps with a little noise
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    X11 = np.stack([(xx - w / 2) / 40.0, (yy - h / 2) / 40.0,
                    2.0 + 0.3 * np.sin(xx / 5.0) * np.cos(yy / 7.0)], -1)[None].repeat(b, 0)
    X11 = (X11 * (1 + 0.01 * rng.normal(size=(b, h, w, 1)))).astype(np.float32)
    X21 = (X11 + 0.02 * rng.normal(size=X11.shape)).astype(np.float32)
    D11 = rng.normal(size=(b, h, w, 24)).astype(np.float32)
    D21 = rng.normal(size=(b, h, w, 24)).astype(np.float32)
    idx_init = rng.integers(0, n, size=(b, n)).astype(np.int64)
    # what the stubbed kernels return
    p_stub = (np.stack([xx, yy], -1).reshape(1, n, 2) + rng.uniform(-2.5, 2.5, size=(b, n, 2)))
    p_stub = np.clip(p_stub, [1, 1], [w - 2, h - 2]).astype(np.float32)
    conv_stub = rng.uniform(size=(b, n)) < 0.8

    stub = types.ModuleType("mast3r_slam_backends")
    stub.iter_proj = lambda *a: [torch.from_numpy(p_stub.copy()), torch.from_numpy(conv_stub)]
    stub.refine_matches = lambda D11, D21, p1, r, d: [p1.clone()]
    sys.modules["mast3r_slam_backends"] = stub
    sys.path.insert(0, REF)
    from mast3r_slam import matching  # noqa: E402
    from mast3r_slam.config import config  # noqa: E402
    config["matching"] = dict(max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6,
                              dist_thresh=1e-1, radius=3, dilation_max=5)

    tX11, tX21 = torch.from_numpy(X11), torch.from_numpy(X21)
    rwg, pts, p_init = matching.prep_for_iter_proj(tX11, tX21, None)
    rwg2, pts2, p_init2 = matching.prep_for_iter_proj(tX11, tX21, torch.from_numpy(idx_init))
    idx, valid = matching.match_iterative_proj(tX11, tX21, torch.from_numpy(D11),
                                               torch.from_numpy(D21), None)
    np.savez_compressed(
        OUT, X11=X11, X21=X21, idx_init=idx_init, p_stub=p_stub, conv_stub=conv_stub,
        rays_with_grad=rwg.numpy(), pts3d_norm=pts.numpy(), p_init=p_init.numpy(),
        p_init_from_idx=p_init2.numpy(), idx=idx.numpy(), valid=valid.numpy())
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
