"""GPU: the per-frame tracking glue of FrameTracker2.track (tracker2.py:127-270) over a
synthetic sequence (analytic pointmaps instead of the random-weight ViT):
frame t is tracked against the keyframe with the previous frame's matches as the
iterative-projection seed (tracker2.py:127), the keyframe pointmap is fused frame after
frame, and every per-frame result is compared with the numpy/C oracle of the same glue
(oracle/frontend_ref.py): match indices and validity bit-exact, poses |dT| <= 1e-4, fused
keyframe pointmap / confidence / count and the lost / new-keyframe decisions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
H, W = 96, 128


def _frames(T=6, seed=0):
    from monst3r_slam_amd import synthetic as syn
    rng = np.random.default_rng(seed)
    out = []
    for t in range(T):
        X11, X21, D11, D21 = syn.pair(H, W, seed=seed + t, shift_px=(0.6 + 0.3 * t, -0.4 + 0.2 * t))
        X = np.stack([X11, X21]).astype(np.float32)
        C = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, H, W)))).astype(np.float32)
        Q = (1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, H, W)))).astype(np.float32)
        if t == 3:
            Q[:] = 1.2      # all Qk <= Q_conf: match_frac 0 → the frame is lost
        D = np.stack([D11, D21]).astype(np.float16)
        out.append((X, C, D, Q))
    return out


def _snapshot_matches(loop):
    """SequenceLoop writes a frame's matches into the tracker's idx_f2k buffer in place (the
    next frame's seed) and its advance resets that buffer to the identity on a keyframe
    replacement: keep a copy of the frame's matches, taken on the stream before advance."""
    adv = loop.advance

    def advance(res, out, feat_i):
        res["idx_match"] = loop.tr.idx_f2k.reshape(-1).clone()   # [1, n] buffer → [n]
        adv(res, out, feat_i)
    loop.advance = advance


def test_tracking_sequence_vs_oracle(dev):
    from monst3r_slam_amd import synthetic as syn
    from monst3r_slam_amd.config import default_config
    from monst3r_slam_amd.frontend import Tracker
    from oracle import frontend_ref as FR
    cfg = default_config()
    frames = _frames()
    Xk0 = syn.backproject(syn.depth_surface(H, W, 5), syn.intrinsics(H, W)).reshape(-1, 3)
    Ck0 = np.full((H * W, 1), 2.0, np.float32)
    Tk = np.array([0.1, -0.05, 0.02, 0, 0, 0, 1, 1.0], np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    tr = Tracker(model=None, cfg=cfg)
    tr.add_keyframe(None, t(Tk), X=t(Xk0.astype(np.float32)), C=t(Ck0),
                    feat=torch.zeros(1, device=dev))
    kf_ref = FR.Keyframe(Xk0, Ck0, Tk)
    idx_ref = None
    for step, (X, C, D, Q) in enumerate(frames):
        out = dict(X=t(X), C=t(C), D16=t(D), Q=t(Q))
        res = tr.track_outputs(out)
        ref = FR.track_outputs(X, C, D, Q, kf_ref, idx_ref, cfg["matching"], cfg["tracking"])
        idx_ref = ref["idx"][None]
        torch.cuda.synchronize()
        assert np.array_equal(res["idx_f2k"].cpu().numpy(), ref["idx"]), step
        assert np.array_equal(res["valid_match"].cpu().numpy(), ref["valid"]), step
        assert bool(res["lost"]) == ref["lost"], step
        if ref["lost"]:
            assert step == 3
        else:
            dT = np.abs(res["T_WCf"].cpu().numpy() - ref["T_WCf"]).max()
            assert dT <= 1e-4, (step, dT)
            assert bool(res["new_kf"]) == ref["new_kf"], step
        np.testing.assert_allclose(tr.kf.X_canon.cpu().numpy(), kf_ref.X_canon, rtol=1e-4,
                                   atol=1e-5)
        np.testing.assert_allclose(tr.kf.C.cpu().numpy(), kf_ref.C, rtol=1e-6)
        assert float(tr.kf.N) == kf_ref.N, step


def test_frame_pipeline_matches_serial_tracking(dev):
    """FramePipeline (next frame's encoder prefetched on a side stream, feature double
    buffer) gives bit-identical per-frame results to Tracker.track on the same frames,
    eager and replayed from the two parity graphs."""
    from monst3r_slam_amd import model as Mdl
    from monst3r_slam_amd.frontend import FramePipeline, Tracker
    m, _ = Mdl.build(dev, small=True)
    Hs, Ws = 96, 128
    g = torch.Generator(device=dev).manual_seed(31)
    imgs = [torch.rand(1, 3, Hs, Ws, device=dev, generator=g) * 2 - 1 for _ in range(5)]
    T0 = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1], dtype=torch.float32, device=dev)

    def run(pipelined):
        tr = Tracker(m)
        tr.add_keyframe(imgs[0], T0)
        out = []
        pipe = FramePipeline(tr, (Hs, Ws)) if pipelined else None
        if pipe:
            pipe.prime(imgs[1], 1)
        for k in range(1, 4):
            r = pipe.step(imgs[k], imgs[k + 1], k) if pipe else tr.track(imgs[k])
            out.append((r["T_WCf"].clone(), r["idx_f2k"].clone(), r["valid_match"].clone(),
                        r["pair"]["X"].clone()))
        torch.cuda.synchronize()
        return out

    a, b = run(False), run(True)
    for k, (ra, rb) in enumerate(zip(a, b)):
        for x, y in zip(ra, rb):
            assert torch.equal(x, y), k


def test_c3_sequence_384x512_vs_oracle(dev, parity_log):
    """configs[2] at its real size: 32 tracked 384x512 frames of the synthetic room sequence
    (monst3r_slam_amd.sequence) through SequenceLoop — stand-in pair outputs, matching seeded
    by the previous frame, pose solve from the previous pose, keyframe fusion, keyframe
    replacement + idx_f2k reset on new_kf, a planted unusable frame (lost) — compared frame
    by frame with the numpy/C oracle of the same main loop (oracle.frontend_ref
    .SequenceOracle): match indices / validity bit-exact, lost / new-keyframe decisions
    equal, |dT_WCf| <= 1e-4, the keyframe state (fused or replaced) within the glue test's
    tolerances.  The sequence must actually replace its keyframe and lose the planted frame."""
    from monst3r_slam_amd import sequence as S
    from monst3r_slam_amd.config import default_config
    from monst3r_slam_amd.frontend import Tracker
    from oracle import frontend_ref as FR
    cfg = default_config()
    F, lost_at = 33, 12
    seq = S.SyntheticSequence(F, 384, 512, device=dev, period=100, lost_frames=(lost_at,))
    tr = Tracker(model=None, cfg=cfg)
    loop = S.SequenceLoop(tr, seq)
    _snapshot_matches(loop)
    loop.reset()
    T0 = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    o = FR.SequenceOracle(seq.Xcam[0].cpu().numpy(), seq.C_own[0].reshape(-1, 1).cpu().numpy(),
                          T0, cfg)
    n_new, n_lost, dT_max = 0, 0, 0.0
    for f in range(1, F):
        res = loop.step()
        out = res["pair"]
        X, C = out["X"].cpu().numpy(), out["C"].cpu().numpy()
        D16, Q = out["D16"].cpu().numpy(), out["Q"].cpu().numpy()
        ref = o.step(X, C, D16, Q)
        assert np.array_equal(res["idx_match"].cpu().numpy(), ref["idx"]), f
        assert np.array_equal(res["valid_match"].cpu().numpy(), ref["valid"]), f
        lost, new_kf = bool(res["lost"]), bool(res["new_kf"])
        assert lost == ref["lost"] and new_kf == ref["new_kf"], f
        assert lost == (f == lost_at), f
        n_new += new_kf
        n_lost += lost
        if not lost:
            dT = float(np.abs(res["T_WCf"].cpu().numpy() - ref["T_WCf"]).max())
            dT_max = max(dT_max, dT)
            assert dT <= 1e-4, (f, dT)
        np.testing.assert_allclose(tr.kf.X_canon.cpu().numpy(), o.kf.X_canon, rtol=1e-4,
                                   atol=1e-5)
        np.testing.assert_allclose(tr.kf.C.cpu().numpy(), o.kf.C, rtol=1e-6)
        assert float(tr.kf.N) == o.kf.N, f
        np.testing.assert_allclose(tr.kf.T_WC.cpu().numpy(), o.kf.T_WC, atol=1e-4)
        if new_kf:   # idx_f2k reset to the identity for the next frame
            assert np.array_equal(tr.idx_f2k[0].cpu().numpy(), np.arange(384 * 512))
    assert n_new >= 1 and n_lost == 1
    summ = loop.summary()
    assert summ["keyframes_added"] == n_new and summ["lost"] == 1
    ate = S.ate_vs_gt(summ["T_WC"][summ["log"][:, 2] == 0],
                      seq.T_gt_np[1:][summ["log"][:, 2] == 0])
    assert ate < 5e-3, ate
    parity_log("test_c3_sequence_384x512_vs_oracle", frames=F - 1, new_keyframes=n_new,
               lost=1, idx_valid="bit-exact", max_abs_dT=dT_max, tol_dT=1e-4, ate_m=ate,
               gn_iterations_hist=summ["gn_iterations_hist"])


def test_c3_sequence_200_pipelined_vs_oracle(dev, parity_log):
    """The headline workload end to end (BASELINE configs[2] as bench.py runs it): all 200
    frames of the synthetic 384x512 room sequence through SequenceLoop with the full-size
    models and the prefetching FramePipeline (the next frame's encoder on a side stream,
    feature double buffer), the stand-in pair outputs, matching, pose solve, keyframe fusion
    and every keyframe replacement — each frame checked against the numpy/C oracle of the
    same main loop: match indices / validity bit-exact, lost / new-keyframe decisions equal,
    |dT_WCf| <= 1e-4, keyframe state within the 32-frame test's tolerances.  The oracle is
    re-seeded each frame with the GPU's incoming state (pose seed, keyframe pose, pointmap,
    confidence, count, match seed): the pose solve stops at |dcost/cost| < 1e-3 or
    |tau| < 1e-3 (tracker2.py:299-357), so a 1e-5 difference in the seed moves the converged
    pose by up to ~1e-4 and 200 chained frames drift apart by more than any per-frame error
    (the chained, unseeded comparison is test_c3_sequence_384x512_vs_oracle, 32 frames).  Every 20th
    frame, the prefetched features must be bit-identical to an encode of the NEXT frame's
    image (the side stream's gather of the frame counter is ordered before the main
    stream's advance rewrites it)."""
    import bench
    from monst3r_slam_amd import sequence as S
    from monst3r_slam_amd.config import default_config
    from monst3r_slam_amd.frontend import FramePipeline
    from oracle import frontend_ref as FR
    cfg = default_config()
    model, tr, seq = bench.setup(dev, 0, bench.SEQ_FRAMES + 1)
    pipe = FramePipeline(tr, (seq.h, seq.w), group=2)   # bench.py's default schedule
    loop = S.SequenceLoop(tr, seq, pipe)
    _snapshot_matches(loop)
    loop.reset(parity=0)
    T0 = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    o = FR.SequenceOracle(seq.Xcam[0].cpu().numpy(), seq.C_own[0].reshape(-1, 1).cpu().numpy(),
                          T0, cfg)
    n_new, dT_max, n_feat = 0, 0.0, 0
    for i in range(bench.SEQ_FRAMES):
        f = i + 1
        # the GPU's incoming state → the oracle (see docstring)
        o.T_prev = loop.T_prev.cpu().numpy().copy()
        o.kf.T_WC = tr.kf.T_WC.cpu().numpy().reshape(8).copy()
        o.kf.X_canon = tr.kf.X_canon.cpu().numpy().copy()
        o.kf.C = tr.kf.C.cpu().numpy().copy()
        o.kf.N = float(tr.kf.N)
        o.idx = tr.idx_f2k.cpu().numpy().copy()
        res = loop.step(i)
        out = res["pair"]
        X, C = out["X"].cpu().numpy(), out["C"].cpu().numpy()
        D16, Q = out["D16"].cpu().numpy(), out["Q"].cpu().numpy()
        ref = o.step(X, C, D16, Q)
        assert np.array_equal(res["idx_match"].cpu().numpy(), ref["idx"]), f
        assert np.array_equal(res["valid_match"].cpu().numpy(), ref["valid"]), f
        lost, new_kf = bool(res["lost"]), bool(res["new_kf"])
        assert lost == ref["lost"] and new_kf == ref["new_kf"], f
        n_new += new_kf
        if not lost:
            dT = float(np.abs(res["T_WCf"].cpu().numpy() - ref["T_WCf"]).max())
            dT_max = max(dT_max, dT)
            assert dT <= 1e-4, (f, dT)
        np.testing.assert_allclose(tr.kf.X_canon.cpu().numpy(), o.kf.X_canon, rtol=1e-4,
                                   atol=1e-5)
        np.testing.assert_allclose(tr.kf.C.cpu().numpy(), o.kf.C, rtol=1e-6)
        assert float(tr.kf.N) == o.kf.N, f
        if i % 20 == 19 and f + 2 < seq.n_frames:
            # the odd step completed the pair that the next two steps track (frames f + 1,
            # f + 2): bit-identical to one two-frame encode of those images (same launches)
            torch.cuda.synchronize()
            got = pipe.pairs[(i // 2 + 1) % 2].clone()
            imgs = seq.img[f + 1:f + 3].reshape(2, 3, seq.h, seq.w)
            assert torch.equal(got, model.encode(imgs, concurrent=True)[0]), f
            imgs = seq.img[f:f + 2].reshape(2, 3, seq.h, seq.w)
            assert not torch.equal(got, model.encode(imgs, concurrent=True)[0]), f
            n_feat += 1
    summ = loop.summary()
    assert summ["keyframes_added"] == n_new >= 2
    ate = S.ate_vs_gt(summ["T_WC"][summ["log"][:, 2] == 0],
                      seq.T_gt_np[1:][summ["log"][:, 2] == 0])
    assert ate < 5e-2, ate
    parity_log("test_c3_sequence_200_pipelined_vs_oracle", frames=bench.SEQ_FRAMES,
               new_keyframes=n_new, idx_valid="bit-exact", max_abs_dT=dT_max, tol_dT=1e-4,
               ate_m=ate, prefetched_features_checked=n_feat,
               gn_iterations_hist=summ["gn_iterations_hist"])


@pytest.mark.parametrize("group", [3, 4])
def test_grouped_prefetch_encodes_the_right_frames(dev, group):
    """FramePipeline(group=g) through SequenceLoop: every completed g-frame group of
    prefetched features equals one direct g-frame encode of exactly the frames the next g
    steps track (part 0 gathers frames t + g .. t + 2g - 1, part g - 1 writes the buffer),
    over two full periods replayed from the captured step graphs."""
    import bench
    from monst3r_slam_amd import sequence as S
    from monst3r_slam_amd.frontend import FramePipeline
    model, tr, seq = bench.setup(dev, 0, 6 * group + 2)
    pipe = FramePipeline(tr, (seq.h, seq.w), group=group)
    loop = S.SequenceLoop(tr, seq, pipe)
    loop.reset(parity=0)
    graphs = [bench.capture(lambda k=k: loop.step(k), dev) for k in range(pipe.period)]
    loop.reset(parity=0)
    torch.cuda.synchronize()
    checked = 0
    for i in range(2 * pipe.period):
        graphs[i % pipe.period].replay()
        if i % group == group - 1:
            torch.cuda.synchronize()
            f0 = i + 2                         # first frame the next group of steps tracks
            got = pipe.pairs[(i // group + 1) % 2].clone()
            imgs = seq.img[f0:f0 + group].reshape(group, 3, seq.h, seq.w)
            assert torch.equal(got, model.encode(imgs, concurrent=True)[0]), i
            checked += 1
    assert checked == 2 * pipe.period // group


def test_c3_sequence_200_graph_replay_equals_eager(dev, parity_log):
    """The bench's timed path is the captured step graphs replayed frame after frame
    (bench.run_sequence); the oracle tests step eagerly.  This closes the gap: all 200 frames
    run eagerly (loop.step) and then from the captured graphs (the bench's capture, stream
    topology checked) — the per-frame log (GN iterations, new-keyframe / lost decisions,
    keyframe frame, T_WC) and the final keyframe state / match seed are bit-identical.  The
    step captures three streams (capture, prefetch, decoder + heads side chain)."""
    import bench
    from monst3r_slam_amd import sequence as S
    from monst3r_slam_amd.frontend import FramePipeline
    model, tr, seq = bench.setup(dev, 0, bench.SEQ_FRAMES + 1)
    tr.split_heads = True
    pipe = FramePipeline(tr, (seq.h, seq.w), group=2)
    loop = S.SequenceLoop(tr, seq, pipe)

    def snap():
        torch.cuda.synchronize()
        return (loop.log_i.clone(), loop.log_T.clone(), tr.kf.X_canon.clone(), tr.kf.C.clone(),
                tr.kf.T_WC.clone(), tr.idx_f2k.clone())

    loop.reset(parity=0)
    for i in range(bench.SEQ_FRAMES):
        loop.step(i % pipe.period)
    eager = snap()
    loop.reset(parity=0)
    graphs = [bench.capture(lambda k=k: loop.step(k), dev) for k in range(pipe.period)]
    assert all(g.m3s_streams == 3 for g in graphs), [g.m3s_streams for g in graphs]
    bench.run_sequence(loop, graphs, bench.SEQ_FRAMES, dev, 1)
    replay = snap()
    names = ("log_i", "log_T", "X_canon", "C", "T_WC", "idx_f2k")
    for nm, a, b in zip(names, eager, replay):
        assert torch.equal(a, b), nm
    summ = loop.summary()
    assert summ["keyframes_added"] >= 2
    parity_log("test_c3_sequence_200_graph_replay_equals_eager", frames=bench.SEQ_FRAMES,
               keyframes_added=summ["keyframes_added"], equal="bit-identical",
               capture_streams=graphs[0].m3s_streams)


def test_malformed_capture_raises_not_crashes(dev):
    """capture.capture_graph checks the fork / join topology on the eager warm-up run, before
    any capture begins: a side stream forked from the capture stream and never joined back
    raises TopologyError (the HIP runtime segfaulted at capture_end on malformed / over-wide
    captures); the same fn with the join captures and replays."""
    from monst3r_slam_amd.capture import TopologyError, capture_graph
    x = torch.zeros(1 << 16, device=dev)
    side = torch.cuda.Stream(dev)

    def unjoined():
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            x.add_(1.0)

    def joined():
        unjoined()
        torch.cuda.current_stream(dev).wait_stream(side)

    with pytest.raises(TopologyError, match="not joined"):
        capture_graph(unjoined, dev)
    torch.cuda.synchronize()
    g = capture_graph(joined, dev)
    assert g.m3s_streams == 2
    before = float(x[0])
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == before + 1.0
