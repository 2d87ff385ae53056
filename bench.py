"""Headline benchmark: tracking frames/sec @512x384 (+ pairwise pointmap-inference ms) on
one MI355X — BASELINE.json metric; workload configs[1]+[2] (bf16 ViT pair inference inside
the full tracking step).

One "step" = one tracked frame of the per-frame hot path, synthetic 384x512 input,
seeded random weights (no checkpoints offline), everything resident in HBM:
  pair inference  MonST3R encoder (new frame) + MonST3R decoder + 2 DPT heads +
                  MASt3R decoder + 2 catmlp+DPT heads (keyframe features cached)
  matching        prep + iter_proj + occlusion + refine_matches + linear index
  tracking        glue (Qk, valid, pointmap fusion, keyframe test) + fused Sim3 GN (≤50 it)
The step is captured once in a HIP graph and replayed (no host work per frame).
Multi-GPU: tracking is sequential per sequence → one independent replica per rank
("replicas only"); value = frames of all ranks / max rank time.

Also measured at every N (field "keyframe_graph", configs[3]): 16 keyframes,
64 pairs re-inferred symmetrically (4 directed decodes + 8 heads each) and matched both ways,
edges sharded round-robin over the ranks with one RCCL all-gather of the per-edge records,
keyframe encoding sharded likewise, then the factor-graph acceptance and the GPU GN solve
(identical on every rank).  value = pairs/s of the whole job (max-over-ranks time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--eager]
                       [--no-graph] [--graph-steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "monst3r-slam_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

H, W = 384, 512
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BF16_DENSE_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (spec, no sparsity)
FP8_DENSE_TFLOPS = 5000.0    # MI355X dense fp8 MFMA (spec, no sparsity; scaled 32x32x64)
METRIC = "tracking frames/sec @512x384 + pairwise pointmap-inference ms, 1/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP graph (debug)")
    ap.add_argument("--no-graph", action="store_true", help="skip the keyframe-graph (C4) leg")
    ap.add_argument("--graph-steps", type=int, default=2)
    ap.add_argument("--no-c5", action="store_true", help="skip the fp8 512x512 dyn-mask leg")
    ap.add_argument("--no-retrieval", action="store_true",
                    help="skip the keyframe-retrieval (loop-closure candidate) leg")
    ap.add_argument("--main-priority", type=int, default=0, help="tracking-chain stream priority")
    ap.add_argument("--side-priority", type=int, default=0, help="prefetch stream priority")
    ap.add_argument("--no-split-heads", action="store_true",
                    help="run the MASt3R DPT heads batched on the tracking chain")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="encode each frame inside its own step (no next-frame encoder overlap)")
    ap.add_argument("--streams", action="store_true",
                    help="overlap independent chains on side streams (measured slower)")
    return ap.parse_args()


def setup(dev, seed):
    """Model (seeded random weights), the synthetic frame / keyframe images, and the
    tracking inputs.  The ViT runs on the images; its random-weight pointmaps carry no
    geometry (no valid matches: every frame would be 'lost' after one GN iteration), so
    matching, the Sim3 GN and the keyframe fusion run on the analytic 384x512 pointmaps /
    descriptors of the synthetic scene (synthetic.pair) against a keyframe displaced by a
    known Sim3 — the tracker does its real iterations every frame."""
    import numpy as np
    from monst3r_slam_amd import model as Mdl
    from monst3r_slam_amd import synthetic as syn
    from monst3r_slam_amd.frontend import Tracker
    model, _ = Mdl.build(dev)
    g = torch.Generator(device=dev).manual_seed(100 + seed)
    img_k = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
    img_f = torch.rand(1, 3, H, W, device=dev, generator=g) * 2 - 1
    rng = np.random.default_rng(seed)
    X11, X21, D11, D21 = syn.pair(H, W, seed=seed, shift_px=(1.5, -0.75))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    glue = dict(X=t(np.stack([X11, X21])),
                C=t((1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, H, W)))).astype(np.float32)),
                D16=t(np.stack([D11, D21]).astype(np.float16)),
                Q=t((1.0 + np.exp(rng.normal(1.0, 0.5, size=(2, H, W)))).astype(np.float32)))
    T_true = np.array([0.02, -0.01, 0.03, *syn.quat_from_axis_angle([0.3, 1.0, 0.2], 0.02), 1.0],
                      np.float32)
    Xk = t(syn.sim3_act(T_true, X21).reshape(-1, 3))
    Ck = torch.full((H * W, 1), 2.0, device=dev)
    tr = Tracker(model)
    T0 = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1], dtype=torch.float32, device=dev)
    feat_k = model.encode(img_k)[0].clone()
    tr.add_keyframe(img_k, T0, X=Xk, C=Ck, feat=feat_k)
    return model, tr, img_f, glue


def capture(fn, dev, priority=0):
    s = torch.cuda.Stream(dev, priority=priority)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    torch.cuda.synchronize(dev)
    return g


def time_replays(g, dev, n):
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def gemm_replay(model, run, dev, reps=20):
    """Average duration of the GEMM launches of one run(): the launches are recorded
    (descriptors, same buffers, same order) during an eager run, captured back-to-back in
    one HIP graph, and that graph is timed with HIP events on the stream it replays on;
    ms / launch is directly comparable to rocprofv3's per-kernel durations of the same
    launches (kernels back to back, as in the step graph).  Returns per-class totals."""
    ops = model.ops
    ops.record = []
    run()
    torch.cuda.synchronize(dev)
    rec, ops.record = ops.record, None
    out = {}
    for name, sel in (("all", lambda r: True), ("fp8", lambda r: r[2])):
        sub = [r for r in rec if sel(r)]
        if not sub:
            continue
        g = capture(lambda sub=sub: [ops.replay_gemm(r[0]) for r in sub], dev)
        ms = time_replays(g, dev, reps)
        fl = sum(r[1] for r in sub)
        out[name] = dict(launches=len(sub), gemm_ms=ms, gemm_flops=fl,
                         avg_launch_us=ms / len(sub) * 1e3, tflops=fl / (ms * 1e-3) / 1e12)
        del g
    return out


def gemm_roofline(model, img, feat_k, dev):
    """GEMM launches of one pair inference (serial schedule), replayed back-to-back."""
    serial, model.serial = model.serial, True
    r = gemm_replay(model, lambda: model.pair(img, feat_j=feat_k), dev)["all"]
    model.serial = serial
    return r


class _Bound:
    """Model handle (monst3r_utils.ModelHandle interface) over the bench's PairModel."""

    def __init__(self, pm):
        self._pm = pm

    def pair_model(self):
        return self._pm


def graph_pairs(n_kf=16, n_pairs=64):
    """Consecutive edges first, then 'retrieval-like' strides, until n_pairs."""
    ii, jj = [], []
    for d in (1, 2, 3, 4, 8, 5, 6, 7):
        for k in range(n_kf - d):
            if len(ii) < n_pairs:
                ii.append(k)
                jj.append(k + d)
    return ii, jj


def keyframe_graph_bench(model, dev, world, steps, warmup=1):
    """configs[3]: sharded 64-pair symmetric re-inference + matching + GN over 16 keyframes."""
    import numpy as np
    from monst3r_slam_amd import global_opt as GO
    from monst3r_slam_amd import parallel as P
    from monst3r_slam_amd import synthetic as syn
    n_kf = 16
    ii, jj = graph_pairs(n_kf, 64)
    sc = syn.keyframe_graph(P=n_kf, h=H, w=W, seed=3)
    g = torch.Generator(device=dev).manual_seed(7)     # same images on every rank
    imgs = torch.rand(n_kf, 1, 3, H, W, device=dev, generator=g) * 2 - 1
    frames = GO.Keyframes(H, W, buffer=n_kf, device=dev)
    frames.img[:n_kf] = imgs
    frames.X[:n_kf] = torch.from_numpy(sc["Xs"]).to(dev)
    frames.C[:n_kf] = torch.from_numpy(sc["Cs"]).to(dev)
    frames.N[:n_kf] = 1
    frames.img_true_shape[:n_kf] = torch.tensor([[H, W]], dtype=torch.int32, device=dev)
    frames.n_size = n_kf
    T0 = torch.from_numpy(sc["Twc"]).to(dev).reshape(n_kf, 1, 8)
    h = _Bound(model)
    group = None

    def step():
        frames.T_WC[:n_kf] = T0
        P.shard_keyframe_features(frames, range(n_kf), model.encode, group)
        graph = P.ShardedFactorGraph(h, h, frames, device=dev, group=group)
        graph.add_factors(ii, jj, min_match_frac=0.0)
        graph.solve_GN_rays()
        return graph

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        graph = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    n = H * W
    del np
    return {"workload": "configs[3]: 16 keyframes, 64 pairs symmetric re-inference (MonST3R+"
                        "MASt3R, 4 decodes + 8 heads each) + 128 directed matches + GN rays",
            "pairs_per_s": len(ii) * steps / el, "ms_per_graph": el / steps * 1e3,
            "steps": steps, "edges_accepted": int(graph.ii.numel()),
            "gflop_per_pair": 3603.6, "tflops_achieved": len(ii) * 3603.6e9 * steps / el / 1e12,
            "allgather_bytes_per_rank": int(-(-len(ii) // world) * P.record_bytes(n)),
            "sharding": f"edges round-robin over {world} rank(s), RCCL all-gather"}


def c5_bench(model, dev, steps):
    """configs[4], one GPU: the per-frame inference of dynamic-mask tracking
    at 512x512 with the fp8 transformer path — MonST3R encoder (new frame), MonST3R-only
    mono decode + both heads (depth for the ego flow), ego flow + flow-error mask (the RAFT
    flow is an input: synthetic here, RAFT is absent code), MonST3R+MASt3R pair decode + 4
    heads + local features vs the cached keyframe, apply_dynamic_mask on C/Q/D.  Graph
    captured; timed for fp8 and for the bf16 path on the same inputs.  Multi-GPU: frames
    are sequential per sequence → replicas (the 1→8 curve is the replica sweep)."""
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import synthetic as syn
    H5 = W5 = 512
    gh = gw = H5 // 16
    g = torch.Generator(device=dev).manual_seed(55)
    img = torch.rand(1, 3, H5, W5, device=dev, generator=g) * 2 - 1
    img_k = torch.rand(1, 3, H5, W5, device=dev, generator=g) * 2 - 1
    K = torch.from_numpy(syn.intrinsics(H5, W5)).to(dev)
    Ti = torch.tensor([0.05, 0.0, 0.01, 0, 0, 0, 1, 1.0], device=dev)
    Tk = torch.tensor([0.0, 0.0, 0.0, 0, 0, 0, 1, 1.0], device=dev)
    flow = torch.randn(2, H5, W5, device=dev, generator=g)
    res = {}
    for mode in ("fp8", "bf16"):
        model.set_fp8(mode == "fp8")
        feat_k = model.encode(img_k)[0].clone()

        def step():
            feat_i, pos = model.encode(img)
            Xm, _ = model.mono(feat_i, H5, W5)
            sR, t = U.sim3_relative_matrix(Ti, Tk)
            ego = U.ego_flow(Xm[0], sR, t, K, K)
            mask = U.dynamic_mask_from_flow(flow, ego, 0.35)
            hooks = model.decode(feat_i[0], feat_k[0], pos, gh, gw)
            pts, conf, d16, d32, dq = model.heads(hooks, gh, gw, H5, W5)
            return U.apply_dynamic_mask_to_pointmaps(pts[0:2], conf[0:2], mask, d16, dq)

        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        gph = capture(step, dev)
        res[mode] = time_replays(gph, dev, steps)
        if mode == "fp8":
            rep = gemm_replay(model, step, dev)
        del gph
    model.set_fp8(False)
    return {"workload": "configs[4]: 512x512 frame, fp8 encoder+decoders, mono decode + ego "
                        "flow + flow-error mask + pair decode/heads + apply_dynamic_mask",
            "ms_per_frame_fp8": res["fp8"], "ms_per_frame_bf16": res["bf16"],
            "frames_per_s_fp8": 1e3 / res["fp8"], "speedup_vs_bf16": res["bf16"] / res["fp8"],
            "fp8_gemm": {"launches": rep["fp8"]["launches"], "ms": rep["fp8"]["gemm_ms"],
                         "gflop": rep["fp8"]["gemm_flops"] / 1e9, "tflops": rep["fp8"]["tflops"],
                         "peak": FP8_DENSE_TFLOPS,
                         "frac": rep["fp8"]["tflops"] / FP8_DENSE_TFLOPS,
                         "timing": "fp8 GEMM launches of one frame replayed back-to-back "
                                   "(HIP graph, HIP events)"},
            "all_gemm_ms": rep["all"]["gemm_ms"],
            "tolerance": "tests/test_gpu_vit.py::test_fp8_model_vs_fp32_restatement_512"}


def retrieval_bench(dev, steps, n_db=64, cpu=True):
    """RetrievalDatabase.update (query + add) per new keyframe at the
    reference's sizes — 768 encoder tokens x 1024, nfeat 300, 64k x 1024 codebook, 5-way query
    assignment — against a database of n_db keyframes, through the public update() (with its
    two host syncs: the entry count and the k returned indices).  The dominant kernel
    (m3s_retr_quantize, 2*300*65536*1024 flop fp32) is timed alone with HIP events on its stream.
    CPU: the numpy oracle's update on the same database size (one keyframe, host cores)."""
    import numpy as np
    from monst3r_slam_amd import _lib
    from monst3r_slam_amd.retrieval import RetrievalDatabase, synthetic_retrieval_weights
    w = synthetic_retrieval_weights(seed=0)
    db = RetrievalDatabase(w, device=dev, image_capacity=n_db + steps + 8)
    g = torch.Generator(device=dev).manual_seed(21)
    feats = [torch.randn(1, 768, 1024, device=dev, generator=g).bfloat16()
             for _ in range(n_db + steps + 2)]
    for f in feats[:n_db]:
        db.update(f, True, 3, 5e-3)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for f in feats[n_db:n_db + steps]:
        db.update(f, True, 3, 5e-3)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    # quantize kernel alone
    lib, s = _lib.load(), _lib.stream(dev)
    q = db.prep_features(feats[-1])[0].contiguous()
    M, k = q.shape[0], 5
    qn = torch.empty(M, dtype=torch.float32, device=dev)
    _lib.check(lib.m3s_retr_rownorm(_lib.ptr(q), M, db.dim, 1, _lib.ptr(qn), s), "qn")
    ws = torch.empty(int(lib.m3s_retr_quantize_workspace_bytes(M, db.ncent, k)), dtype=torch.uint8,
                     device=dev)
    codes = torch.empty((M, k), dtype=torch.int32, device=dev)
    reps = 20
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps + 2):
        if r == 2:
            ev0.record()
        _lib.check(lib.m3s_retr_quantize(_lib.ptr(q), _lib.ptr(qn), M, _lib.ptr(db.centroids),
                                         _lib.ptr(db.cnorm2), db.ncent, db.dim, k, _lib.ptr(codes),
                                         None, _lib.ptr(ws), s), "quantize")
    ev1.record()
    torch.cuda.synchronize(dev)
    q_ms = ev0.elapsed_time(ev1) / reps
    flop = 2.0 * M * db.ncent * db.dim
    out = {"workload": f"RetrievalDatabase.update(add_after_query=True, k=3) per keyframe, "
                       f"{n_db}+ keyframes indexed, 768x1024 tokens, nfeat 300, "
                       f"{db.ncent}x{db.dim} codebook, query multiple assignment 5",
           "ms_per_keyframe_update": ms, "updates_per_s": 1e3 / ms,
           "quantize_kernel": {"ms": q_ms, "tflops": flop / q_ms / 1e9, "peak_fp32_vector": 157.3,
                               "frac": flop / q_ms / 1e9 / 157.3,
                               "timing": "HIP events on the launch stream (the current stream)"}}
    if cpu:
        from oracle import retrieval_ref as R
        wn = dict(w)
        ref = R.RetrievalDatabase(wn, w["centroids"])
        # index n_db keyframes cheaply: reuse the GPU's aggregated database contents
        for gi in range(n_db):
            n0, n1 = int(db.img_start[gi]), int(db.img_start[gi + 1])
            ref.ivf.add(db.db_packed[n0:n1].cpu().numpy().view(np.uint32),
                        db.db_words[n0:n1].cpu().numpy(), gi)
        ref.kf_counter = n_db
        f = feats[-2][0].float().cpu().numpy()
        t0 = time.perf_counter()
        ref.update(f, True, 3, 5e-3)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"ms_per_keyframe_update": dt * 1e3, "kind": "port",
                               "cores": torch.get_num_threads(),
                               "sample": "numpy oracle update of one keyframe vs the same "
                                         f"{n_db}-keyframe database (fp64 whitening, fp32 "
                                         "quantisation GEMM, python inverted file)"}
    return out


def pmc_traffic():
    """HBM bytes of the GEMM launches of one pair inference, from the committed rocprofv3
    PMC passes (tools/pmc_traffic.py over FETCH_SIZE / WRITE_SIZE runs of this bench; PMC
    counters cannot be read from inside the timed run).  None if absent."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_gemm_traffic.json")
    if not os.path.exists(path):
        return None
    g = json.load(open(path))["gemm"]
    return g


def cpu_baseline():
    """The reference-equivalent CPU path on this box's host cores, bounded sample:
    the fp32 PyTorch restatement of the pair inference at 224x224 (configs[0] plumbing
    case) scaled by FLOPs to 384x512, plus the C oracle of matching and the
    numpy tracker on one 384x512 frame."""
    import numpy as np
    from monst3r_slam_amd import synthetic as syn
    from monst3r_slam_amd import weights as Wt
    from monst3r_slam_amd.config import default_config
    from oracle import oracle as O
    from oracle import tracker_ref as TR
    from oracle import vit_ref as V
    torch.set_flush_denormal(True)
    nthreads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(nthreads)
    am, aM = Wt.MONST3R, Wt.MAST3R
    sdm = Wt.make_state_dict(am, 0)
    sdM = Wt.make_state_dict(aM, 1)
    g = torch.Generator().manual_seed(1)
    img_i = torch.rand(1, 3, 224, 224, generator=g) * 2 - 1
    img_j = torch.rand(1, 3, 224, 224, generator=g) * 2 - 1
    t0 = time.perf_counter()
    V.asymmetric_inference(sdm, am, sdM, aM, img_i, img_j)
    t_vit224 = time.perf_counter() - t0
    # pair FLOPs 384x512 vs 224x224 (both encoders at 224: one extra encoder pass there)
    scale = 2324.8 / (2324.8 * (196 / 768) + 523.0 * 196 / 768)
    t_vit = t_vit224 * scale
    O.build()
    X11, X21, D11, D21 = syn.pair(H, W, seed=0)
    p = syn.tracking_problem(H, W, seed=0)
    t0 = time.perf_counter()
    O.match(X11[None], X21[None], D11[None], D21[None])
    TR.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"],
                              default_config()["tracking"])
    t_match = time.perf_counter() - t0
    del np
    return {"value": 1.0 / (t_vit + t_match), "unit": "frames/s", "cores": nthreads,
            "kind": "port",
            "sample": f"fp32 torch-CPU pair inference at 224x224 ({t_vit224:.2f} s, scaled by "
                      f"FLOPs x{scale:.2f} to 384x512) + C-oracle matching + numpy tracker GN "
                      f"on one 384x512 frame ({t_match:.2f} s)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    model, tr, img_f, glue = setup(dev, rank)
    model.serial = not args.streams
    tr.split_heads = not args.no_split_heads

    from monst3r_slam_amd.frontend import FramePipeline
    pipe = None if args.no_prefetch else FramePipeline(tr, (H, W), args.side_priority)

    def step(k=0):
        """One tracked frame: pair inference on the frame image (encoder output prefetched
        by the previous step unless --no-prefetch; this step encodes the next frame on the
        side stream), then matching + GN + fusion on the synthetic scene's pointmaps."""
        main = torch.cuda.current_stream(dev)
        feat_i = None
        if pipe is not None:
            pipe.side.wait_stream(main)
            with torch.cuda.stream(pipe.side):
                model.encode(img_f, out=pipe.feat[(k + 1) % 2])   # every frame is img_f
            feat_i = pipe.feat[k % 2]
        out = model.pair(img_f, feat_j=tr.kf.feat, feat_i=feat_i, split_heads=tr.split_heads)
        res = tr.track_outputs(glue)
        model.join()
        if pipe is not None:
            main.wait_stream(pipe.side)
        res["pair"] = out
        return res

    if pipe is not None:
        pipe.prime(img_f, 0)
    for w in range(args.warmup):
        step(2 * w)
    torch.cuda.synchronize(dev)
    # two graphs with the feature double-buffer parities swapped, replayed alternately
    g_steps = None if args.eager else [capture(lambda: step(0), dev, args.main_priority),
                                       capture(lambda: step(1), dev, args.main_priority)]
    g_pair = None if args.eager else capture(lambda: model.pair(img_f, feat_j=tr.kf.feat), dev)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if g_steps is not None:
            g_steps[i % 2].replay()
        else:
            step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        res = step(0)
        gn_info = [int(v) for v in res["info"].tolist()]   # iterations, fail, converged
        pair_ms = time_replays(g_pair, dev, max(5, args.steps // 2)) if g_pair else None
        roof = gemm_roofline(model, img_f, tr.kf.feat, dev)
        pmc = pmc_traffic()
        ms = elapsed / args.steps * 1e3
        line = {
            "metric": METRIC,
            "value": world * args.steps / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded random images and weights, no checkpoints offline; "
                    "matching/GN/fusion on the analytic pointmaps of the synthetic scene)",
            "config": {"workload": "tracking step 384x512: MonST3R+MASt3R pair inference + "
                                   "projective matching + Sim3 ray GN (configs[1]+[2])",
                       "schedule": ("serial" if pipe is None else
                                    "next frame's encoder prefetched on a side stream") +
                                   ("" if args.no_split_heads else
                                    "; MASt3R DPT heads on a side stream"),
                       "h": H, "w": W, "models": "MonST3R ViT-L/B dpt + MASt3R ViT-L/B catmlp+dpt",
                       "parallelism": f"replicas{world}"},
            "pair_inference_ms": pair_ms,
            "tracker_gn": {"iterations": gn_info[0], "fail": gn_info[1], "converged": gn_info[2]},
            "roofline": {"bound": "mfma", "achieved": roof["tflops"], "peak": BF16_DENSE_TFLOPS,
                         "unit": "TFLOP/s", "frac": roof["tflops"] / BF16_DENSE_TFLOPS,
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "traffic_unit": "HBM bytes per GEMM launch (PMC FETCH_SIZE x2 + "
                                         "WRITE_SIZE, profiles/r01_pmc_gemm_traffic.json)",
                         "traffic_per_pair_bytes": pmc["hbm_bytes_per_pair"] if pmc else None,
                         "l2_hit_rate": pmc["l2_hit_rate"] if pmc else None,
                         "kernel": "gemm_kernel (bf16 MFMA GEMM / implicit conv)",
                         "timing": "the pair's GEMM launches replayed back-to-back in one HIP "
                                   "graph, HIP events on its stream (bench.gemm_replay)",
                         "gemm_launches_per_pair": roof["launches"],
                         "gemm_ms_per_pair": roof["gemm_ms"],
                         "gemm_gflop_per_pair": roof["gemm_flops"] / 1e9,
                         "avg_launch_us": roof["avg_launch_us"]},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline()
    if not args.no_c5 and rank == 0:
        line["fp8_dynmask_512"] = c5_bench(model, dev, max(5, args.steps // 2))
    if not args.no_retrieval and rank == 0:
        line["keyframe_retrieval"] = retrieval_bench(
            dev, max(5, args.steps // 2), cpu=not args.no_cpu_baseline and world == 1)
    if not args.no_graph:
        kg = keyframe_graph_bench(model, dev, world, args.graph_steps)
        if rank == 0:
            line["keyframe_graph"] = kg
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
