"""CPU: trajectory outputs (monst3r_slam_amd.evaluate vs mast3r_slam/evaluate.py:24-45,
110-141 and lietorch_utils.as_SE3) — TUM line format, keyframe timestamps by frame_id,
full-trajectory ordering by frame id — and the ATE metric (Umeyama alignment)."""
import types

import numpy as np
import pytest

from monst3r_slam_amd import evaluate as E
from monst3r_slam_amd import synthetic as syn


def _sim3(t, axis, ang, s):
    return np.concatenate([t, syn.quat_from_axis_angle(axis, ang), [s]]).astype(np.float32)


def test_save_traj_format(tmp_path):
    kfs = [types.SimpleNamespace(frame_id=fid, T_WC=_sim3([0.1 * fid, 0.2, -0.3], [0, 1, 0],
                                                          0.05 * fid, 1.5)[None])
           for fid in (0, 4, 9)]
    ts = [float(i) / 30 for i in range(10)]
    E.save_traj(tmp_path / "logs", "seq.txt", ts, kfs)
    lines = open(tmp_path / "logs" / "seq.txt").read().splitlines()
    assert len(lines) == 3
    for ln, kf in zip(lines, kfs):
        v = ln.split()
        assert len(v) == 8 and float(v[0]) == ts[kf.frame_id]
        d = kf.T_WC.reshape(-1)
        # f-string of the numpy f32 scalars, as the reference formats them
        assert v[1:] == [f"{x}" for x in d[:7]]
        np.testing.assert_array_equal(np.float32(v[1:]), d[:7])      # scale dropped (as_SE3)


def test_save_full_traj_sorted_by_frame_id(tmp_path):
    ids = np.array([3, 0, 2, 1])
    ts = ["1305031102.175304", "1305031102.211214", "1305031102.243211", "1305031102.275326"]
    T = np.stack([_sim3([i, 0, 0], [1, 0, 0], 0.0, 2.0) for i in ids])
    E.save_full_traj(tmp_path, "full.txt", ids, ts, T)
    rows = [ln.split() for ln in open(tmp_path / "full.txt")]
    assert [r[0] for r in rows] == [ts[1], ts[3], ts[2], ts[0]]
    assert [float(r[1]) for r in rows] == [0.0, 1.0, 2.0, 3.0]


def test_ate_zero_under_sim3_and_positive_with_noise(tmp_path):
    rng = np.random.default_rng(0)
    n = 50
    t = np.cumsum(rng.normal(size=(n, 3)) * 0.1, 0)
    q = np.tile([0, 0, 0, 1.0], (n, 1))
    ts = np.arange(n) / 30.0
    ref = tmp_path / "ref.txt"
    with open(ref, "w") as f:
        for i in range(n):
            f.write(f"{ts[i]} " + " ".join(str(x) for x in np.r_[t[i], q[i]]) + "\n")
    R = syn.quat_to_rot(syn.quat_from_axis_angle([0.3, 1, 0.2], 0.7))
    est_t = 2.5 * (R @ t.T).T + np.array([1.0, -2.0, 0.5])
    est = tmp_path / "est.txt"
    with open(est, "w") as f:
        for i in range(n):
            f.write(f"{ts[i] + 0.001} " + " ".join(str(x) for x in np.r_[est_t[i], q[i]]) + "\n")
    rmse, m = E.ate(est, ref)
    assert m == n and rmse < 1e-9
    rmse_se3, _ = E.ate(est, ref, with_scale=False)
    assert rmse_se3 > 0.1                      # scale cannot be absorbed without Sim3
    noisy = tmp_path / "noisy.txt"
    with open(noisy, "w") as f:
        for i in range(n):
            p = t[i] + rng.normal(size=3) * 0.01
            f.write(f"{ts[i]} " + " ".join(str(x) for x in np.r_[p, q[i]]) + "\n")
    rmse, _ = E.ate(noisy, ref)
    assert 0.005 < rmse < 0.02


def test_ate_needs_associations(tmp_path):
    a = tmp_path / "a.txt"
    a.write_text("0 0 0 0 0 0 0 1\n")
    with pytest.raises(ValueError):
        E.ate(a, a)
