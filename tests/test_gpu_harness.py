"""GPU: the whole main loop (harness.SlamLoop — main_monster_slam.py:247-332 with the
backend :81-149 and relocalisation :20-78 at the single-thread wait points) on the
synthetic room sequence, every component real (matching, tracker, keyframe store,
FactorGraph + GN, retrieval database) with the perfect-network stand-in for the pair
model (scene_model.SceneModel); and the loop on the real (random-weight, reduced-width)
networks for a few frames, exercising INIT / TRACKING / RELOC on the HIP model path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_synthetic_sequence_ate(dev, tmp_path):
    """TRACKING branch alone (run_tracking) on synthetic.tracking_sequence: ATE < 1 mm,
    per-frame translations within 3 mm (whole-pixel matches vs the frames' 0.3-0.7 px image
    shifts bias each unaligned pose by about 1 mm, as they would the reference's)."""
    from monst3r_slam_amd.harness import synthetic_run
    rmse, lost, T_WC, T_gt = synthetic_run(dev, str(tmp_path), n=8)
    assert not lost.any()
    assert rmse < 1e-3, rmse
    np.testing.assert_allclose(T_WC[:, :3], T_gt[:, :3], atol=3e-3)
    assert len(open(tmp_path / "est.txt").read().splitlines()) == 8


def test_slam_loop_scene_init_track_reloc_keyframes(dev, tmp_path, parity_log):
    from monst3r_slam_amd import harness as Hn
    rmse, loop = Hn.scene_slam_run(dev, str(tmp_path), n=120, h=96, w=128, period=100,
                                   lost_frames=(60,))
    kinds = [e[1] for e in loop.events]
    parity_log("slam_loop_scene_120", ate_m=rmse, keyframes=len(loop.keyframes),
               edges=int(loop.graph.ii.numel()), events=loop.events[:20],
               modes={m: loop.modes.count(m) for m in set(loop.modes)})
    assert loop.modes[0] == "INIT" and loop.modes.count("INIT") == 1
    assert (60, "lost", None) in loop.events
    assert "reloc_ok" in kinds and loop.modes[61] == "RELOC"
    assert kinds.count("new_kf") >= 2 and len(loop.keyframes) >= 4
    assert loop.graph.ii.numel() >= len(loop.keyframes) - 1
    assert np.isfinite(np.stack(loop.poses)).all()
    assert rmse < 0.05, rmse
    # the backend moved no pose off the first keyframe (pin = 1) and kept keyframe 0 at I
    T0 = loop.keyframes.T_WC[0, 0].cpu().numpy()
    np.testing.assert_allclose(T0, [0, 0, 0, 0, 0, 0, 1, 1], atol=1e-6)


def test_slam_loop_on_the_hip_networks(dev, tmp_path):
    from monst3r_slam_amd import harness as Hn
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import retrieval as R
    from monst3r_slam_amd import weights as Wt
    mon = U.load_monst3r(device=dev, arch=Wt.small(Wt.MONST3R))
    mas = U.load_mast3r(device=dev, arch=Wt.small(Wt.MAST3R))
    pm = mon.pair_model()
    h, w = 96, 128
    ret = R.load_retriever(device=dev, weights=R.synthetic_retrieval_weights(
        enc_dim=pm.a.enc_dim, ncent=4096))
    loop = Hn.SlamLoop(pm, mas, mon, h, w, dev, ret)
    g = torch.Generator(device=dev).manual_seed(4)
    base = torch.rand(1, 3, h, w, device=dev, generator=g) * 2 - 1
    imgs = [(base + 0.02 * k).clamp(-1, 1) for k in range(5)]
    T = loop.run(imgs, [str(k) for k in range(5)], str(tmp_path))
    assert loop.modes[0] == "INIT" and set(loop.modes) <= {"INIT", "TRACKING", "RELOC"}
    assert T.shape == (5, 8) and np.isfinite(T).all()
    assert len(loop.keyframes) >= 1
