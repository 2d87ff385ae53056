"""GPU: headless tracking harness (monst3r_slam_amd.harness, main_monster_slam.py:247-332
TRACKING branch) over a synthetic sequence with ground truth: every frame tracked through the
HIP matching + glue + Sim3 GN, the TUM trajectory written by save_full_traj, and the ATE
against the ground-truth file (Sim3-aligned) below 1 mm.  Per-frame translations within
3 mm: matches are whole pixels while the synthetic frames carry sub-pixel image shifts
(0.3-0.7 px), which biases each unaligned pose by about 1 mm, as it would the reference's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_synthetic_sequence_ate(dev, tmp_path):
    from monst3r_slam_amd.harness import synthetic_run
    rmse, lost, T_WC, T_gt = synthetic_run(dev, str(tmp_path), n=8)
    assert not lost.any()
    assert rmse < 1e-3, rmse
    np.testing.assert_allclose(T_WC[:, :3], T_gt[:, :3], atol=3e-3)
    assert len(open(tmp_path / "est.txt").read().splitlines()) == 8
