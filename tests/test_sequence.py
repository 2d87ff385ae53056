"""CPU: the configs[2] synthetic sequence (monst3r_slam_amd.sequence) and the main-loop
oracle over it (oracle.frontend_ref.SequenceOracle) — the GPU test
tests/test_gpu_sequence.py::test_c3_sequence_384x512_vs_oracle compares the HIP loop with
the same oracle frame by frame."""
import numpy as np
import pytest
import torch

from monst3r_slam_amd import sequence as S
from monst3r_slam_amd import synthetic as syn


def _outputs(s, t, j):
    """numpy statement of m3s_seq_pair_outputs (frame t against keyframe j)."""
    H, W = s.h, s.w
    Trel = syn.sim3_mul(syn.sim3_inv(s.T_gt_np[t]), s.T_gt_np[j])
    X = np.stack([s.Xcam[t].numpy(), syn.sim3_act(Trel, s.Xcam[j].numpy())]).reshape(2, H, W, 3)
    C = np.stack([s.C_own[t].numpy(), s.C_other[t].numpy()]).reshape(2, H, W)
    Q = np.stack([s.Q_own[t].numpy(), s.Q_other[t].numpy()]).reshape(2, H, W)
    D = np.stack([s.D16[t].numpy(), s.D16[j].numpy()]).reshape(2, H, W, 24)
    return X.astype(np.float32), C, D, Q


def test_trajectory_and_scene():
    T = S.trajectory(201)
    assert np.allclose(T[0], [0, 0, 0, 0, 0, 0, 1, 1])
    assert np.allclose(np.linalg.norm(T[:, 3:7], axis=1), 1, atol=1e-6)
    assert np.allclose(T[200], T[0], atol=1e-5)          # periodic
    s = S.SyntheticSequence(4, 48, 64, period=20, lost_frames=(2,))
    assert bool((s.Xcam[:, :, 2] > 0.5).all()) and bool(torch.isfinite(s.Xcam).all())
    nrm = s.D16.float().norm(dim=-1)
    assert float((nrm - 1).abs().max()) < 2e-3
    assert float(s.img.min()) >= -1 and float(s.img.max()) <= 1
    assert bool((s.Q_own[2] == 1.2).all())
    # the keyframe's pixels, moved into frame 1's camera, land where frame 1 sees the same
    # surface (non-occluded pixels): reprojection through frame 1's pointmap
    X, _, _, _ = _outputs(s, 1, 0)
    K = s.K
    uv = X[1].reshape(-1, 3) @ K.T
    uv = uv[:, :2] / uv[:, 2:3]
    inside = (uv[:, 0] > 0) & (uv[:, 0] < 63) & (uv[:, 1] > 0) & (uv[:, 1] < 47)
    ui, vi = np.round(uv[inside]).astype(int).T
    d = np.linalg.norm(X[0][vi, ui] - X[1].reshape(-1, 3)[inside], axis=1)
    assert np.median(d) < 0.05


def test_sequence_oracle_tracks_with_keyframe_turnover(oracle):
    from monst3r_slam_amd.config import default_config
    from oracle import frontend_ref as FR
    F = 41
    s = S.SyntheticSequence(F, 96, 128, period=100, lost_frames=(17,))
    o = FR.SequenceOracle(s.Xcam[0].numpy(), s.C_own[0].numpy()[:, None],
                          np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32), default_config())
    j, new, lost, est = 0, 0, [], []
    for t in range(1, F):
        r = o.step(*_outputs(s, t, j))
        lost.append(r["lost"])
        if r["new_kf"]:
            j = t
            new += 1
        est.append(o.T_prev.copy())
    assert [t + 1 for t, lo in enumerate(lost) if lo] == [17]
    assert new >= 1
    ok = ~np.array(lost)
    ate = S.ate_vs_gt(np.array(est)[ok], s.T_gt_np[1:][ok])
    assert ate < 0.02, ate
