"""Per-shape GEMM launch configuration sweep for the pair inference (and the mono / symmetric
decodes when --graph): every recorded launch class (M, N, K, batch, flags, mode) is replayed
back to back in a HIP graph under each (tile, split-K, fused) choice (env overrides read by
m3s_vit_gemm at capture time) and timed with HIP events.  Writes the per-shape best as JSON
and as the C table gemm_table.inc (next to the JSON; copied to monst3r-slam_amd/csrc/)
that m3s_vit_gemm consults before
its heuristic.  Isolated per-launch times are the criterion here; a choice is kept in the
table only if it beats the heuristic by > 3 % — the pipelined step is the final judge
(bench.py), as DESIGN §2 records for the 96-row tiles.

  python tools/gemm_autotune.py [--out gpurun_out/gemm_autotune.json] [--write-table]
"""
import argparse
import collections
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

TILES = {1: "128x128", 2: "64x128 2/CU", 7: "128x128 2/CU", 8: "96x128",
         10: "64x128 6-stage", 11: "128x128 4-stage", 12: "128x128 8 waves", 6: "256x128", 13: "256x128 8 waves"}
SPLITS = (1, 2, 3, 4, 6, 8)


def record(m, dev, graph, split_heads=False, c5=False, fp8=False):
    img = torch.rand(1, 3, 384, 512, device=dev) * 2 - 1
    feat, _ = m.encode(img)
    feat = feat.clone()
    m.ops.record = []
    m.pair(img, feat_j=feat)
    if split_heads:  # the C3 step's head launches (MonST3R / MASt3R heads as two batch-2 sets)
        m.pair(img, feat_j=feat, split_heads=True)
    if c5:  # the configs[4] 512x512 frame's bf16 launches (heads) beside its fp8 ViT
        # (set_fp8 calibrates on two frames through scratch buffers it frees afterwards: its
        # launches are not recorded — replaying their descriptors would touch freed memory;
        # round 6: a recorded calibration conv replayed after the scratch was released
        # faulted with an illegal address)
        rec, m.ops.record = m.ops.record, None
        m.set_fp8(True)
        m.ops.record = rec
        img5 = torch.rand(1, 3, 512, 512, device=dev) * 2 - 1
        f5 = m.encode(img5)[0].clone()
        feat_i, pos = m.encode(img5)
        m.mono(feat_i, 512, 512)
        hooks = m.decode(feat_i[0], f5[0], pos, 32, 32)
        m.heads(hooks, 32, 32, 512, 512)
        m.set_fp8(False)
    if graph:
        m.mono(feat, 384, 512)
        f4 = feat.expand(4, -1, -1).contiguous()
        m.symmetric(f4, f4, 384, 512)
    torch.cuda.synchronize()
    rec, m.ops.record = m.ops.record, None
    groups = collections.OrderedDict()
    for d, fl, f8 in rec:
        if f8 and not fp8:
            continue
        if fp8 and not f8:
            continue
        key = (d.M, d.N, d.K, d.batch, d.flags, d.mode)
        groups.setdefault(key, []).append((d, fl))
    return groups


def time_group(m, dev, lst, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        reps = max(1, 24 // len(lst))
        g = bench.capture(lambda: [m.ops.replay_gemm(d) for d, _ in lst * reps], dev)
        ms = bench.time_replays(g, dev, 5) / (reps * len(lst))
        del g
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return ms * 1e3  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "gemm_autotune.json"))
    ap.add_argument("--write-table", action="store_true")
    ap.add_argument("--graph", action="store_true", help="also the mono / symmetric shapes")
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--tiles", type=lambda v: [int(t) for t in v.split(",")], default=None,
                    help="restrict the sweep to these tile configs")
    ap.add_argument("--gemm-only-m", type=int, default=0, help="only launch classes with this M")
    ap.add_argument("--split-heads", action="store_true", help="also the split-heads pair shapes")
    ap.add_argument("--c5", action="store_true", help="also the 512x512 fp8 frame's bf16 launches")
    ap.add_argument("--fp8", action="store_true", help="with --c5: its fp8 launches instead")
    ap.add_argument("--min-m", type=int, default=0, help="only launch classes with M >= this")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m, _ = Mdl.build(dev)
    for k in ("M3S_GEMM_TILE", "M3S_GEMM_SPLITS", "M3S_GEMM_FUSED"):
        os.environ.pop(k, None)
    groups = record(m, dev, args.graph, args.split_heads, args.c5, args.fp8)
    res = []
    for key, lst in groups.items():
        M, N, K, batch, flags, mode = key
        if args.gemm_only_m and M != args.gemm_only_m:
            continue
        if M < args.min_m:
            continue
        base = time_group(m, dev, lst, {})
        best = (base, None)
        tried = {}
        for tile in TILES:
            if mode == 1 and tile in (8, 10, 11):
                continue
            if args.tiles and tile not in args.tiles:
                continue
            for sp in SPLITS:
                for fu in ((0, 1) if sp > 1 else (0,)):
                    if sp > 1 and tile == 8:
                        continue
                    if mode == 1 and sp > 1 and tile != 2:
                        continue
                    us = time_group(m, dev, lst, {"M3S_GEMM_TILE": tile, "M3S_GEMM_SPLITS": sp,
                                                  "M3S_GEMM_FUSED": fu})
                    tried[f"{tile}/{sp}/{fu}"] = round(us, 2)
                    if us < best[0]:
                        best = (us, (tile, sp, fu))
        fl = sum(f for _, f in lst) / len(lst)
        row = dict(M=M, N=N, K=K, batch=batch, flags=flags, mode=mode, launches=len(lst),
                   base_us=round(base, 2), best_us=round(best[0], 2), best=best[1],
                   base_tflops=fl / base / 1e6, best_tflops=fl / best[0] / 1e6, tried=tried)
        res.append(row)
        print(f"{str(key):44s} n={len(lst):3d} base {base:7.2f} us ({fl / base / 1e6:6.1f} TF/s)"
              f" best {best[0]:7.2f} us {best[1]}", flush=True)
    tot_b = sum(r["base_us"] * r["launches"] for r in res)
    tot_n = sum(r["best_us"] * r["launches"] for r in res)
    print(f"GEMM per recorded run: heuristic {tot_b:.1f} us, best per shape {tot_n:.1f} us")
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(dict(rows=res, total_base_us=tot_b, total_best_us=tot_n), open(args.out, "w"),
              indent=1)
    if args.write_table:
        lines = ["// Generated by tools/gemm_autotune.py (graph-replayed per-launch sweep on MI355X):",
                 "// {M, N, K, batch, flags, mode, tile config, split-K, fused} — shapes whose best",
                 f"// choice beat the heuristic by > {args.min_gain:.0%}.",
                 ]
        for r in res:
            if r["best"] is None or r["best_us"] > (1 - args.min_gain) * r["base_us"]:
                continue
            t, sp, fu = r["best"]
            lines.append(f"{{{r['M']}, {r['N']}, {r['K']}, {r['batch']}, {r['flags']}, {r['mode']}, "
                         f"{t}, {sp}, {fu}}},  // {r['base_us']:.1f} -> {r['best_us']:.1f} us")
        # lands in gpurun_out/ (merged back from the GPU box); copy it to csrc/ and rebuild
        path = os.path.join(os.path.dirname(args.out), "gemm_table.inc")
        open(path, "w").write("\n".join(lines) + "\n")
        print("wrote", path)


if __name__ == "__main__":
    main()
