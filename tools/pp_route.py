"""Which recorded GEMM launch classes the 256x256 ping-pong kernel (T256PP, tile 15) should
take: every launch class of the pair inference (+ the split-heads pair, the mono and
symmetric decodes with --graph, the C5 frame's bf16 launches with --c5) is replayed back to
back in a HIP graph under the current choice (table / heuristic) and under T256PP (unsplit),
timed with HIP events (tools/gemm_autotune.py's method).  Prints per class, and with
--write writes gpurun_out/gemm_table_pp.inc: the current table with the classes where T256PP
wins by > --min-gain switched to it (copy to monst3r-slam_amd/csrc/gemm_table.inc).

  python tools/pp_route.py [--graph] [--c5] [--split-heads] [--write] [--min-m 512]
"""
import argparse
import json
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "monst3r-slam_amd")]
import gemm_autotune as GA  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--c5", action="store_true")
    ap.add_argument("--split-heads", action="store_true")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--min-m", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pp_route.json"))
    ap.add_argument("--sym-pairs", type=lambda v: [int(x) for x in v.split(",") if x],
                    default=[], help="also symmetric decodes of these pair counts (one chunk)")
    ap.add_argument("--encode-batch", type=int, default=0, help="also a batched encode")
    ap.add_argument("--t192", action="store_true", help="also try T192PP (tile 16)")
    ap.add_argument("--only-batch", type=lambda v: [int(x) for x in v.split(",") if x],
                    default=[], help="only launch classes of these batch sizes")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m, _ = Mdl.build(dev)
    for k in ("M3S_GEMM_TILE", "M3S_GEMM_SPLITS", "M3S_GEMM_FUSED"):
        os.environ.pop(k, None)
    groups = GA.record(m, dev, args.graph, args.split_heads, args.c5, False)
    # extra launch classes: symmetric decodes of other chunk sizes (the keyframe graph's
    # near-equal chunks) and a batched keyframe encode (the C4 leg's shard_keyframe_features)
    extra = []
    img = torch.rand(1, 3, 384, 512, device=dev) * 2 - 1
    feat = m.encode(img)[0].clone()
    m.ops.record = []
    for nb in args.sym_pairs:
        f = feat.expand(nb, -1, -1).contiguous()
        m.symmetric(f, f, 384, 512, chunk=nb)
    if args.encode_batch:
        m.encode(torch.rand(args.encode_batch, 3, 384, 512, device=dev) * 2 - 1)
    torch.cuda.synchronize()
    extra, m.ops.record = m.ops.record, None
    for d, fl, f8 in extra:
        if f8:
            continue
        groups.setdefault((d.M, d.N, d.K, d.batch, d.flags, d.mode), []).append((d, fl))
    rows = []
    for key, lst in groups.items():
        M, N, K, batch, flags, mode = key
        if M < args.min_m or (args.only_batch and batch not in args.only_batch):
            continue
        base = min(GA.time_group(m, dev, lst, {}) for _ in range(2))
        # the ping-pong tiles: T256PP (15) and, with --t192, T192PP (16)
        best_pp, pp_cfg = None, 15
        for cfg in ([15, 16] if args.t192 else [15]):
            t = min(GA.time_group(m, dev, lst, {"M3S_GEMM_TILE": cfg, "M3S_GEMM_SPLITS": 1,
                                                "M3S_GEMM_FUSED": 0}) for _ in range(2))
            if best_pp is None or t < best_pp:
                best_pp, pp_cfg = t, cfg
        pp = best_pp
        fl = sum(f for _, f in lst) / len(lst)
        rows.append(dict(M=M, N=N, K=K, batch=batch, flags=flags, mode=mode, launches=len(lst),
                         base_us=round(base, 2), pp_us=round(pp, 2), pp_cfg=pp_cfg,
                         base_tflops=fl / base / 1e6, pp_tflops=fl / pp / 1e6))
        name = "T256PP" if pp_cfg == 15 else "T192PP"
        print(f"{str(key):44s} n={len(lst):3d} current {base:8.2f} us ({fl / base / 1e6:6.1f} "
              f"TF/s)  {name} {pp:8.2f} us ({fl / pp / 1e6:6.1f} TF/s)"
              f"{'  <- PP' if pp < (1 - args.min_gain) * base else ''}", flush=True)
    tb = sum(r["base_us"] * r["launches"] for r in rows)
    tp = sum(min(r["base_us"], r["pp_us"]) * r["launches"] for r in rows)
    print(f"GEMM per recorded run: current {tb:.1f} us, with T256PP where it wins {tp:.1f} us")
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(dict(rows=rows, total_current_us=tb, total_with_pp_us=tp), open(args.out, "w"),
              indent=1)
    if args.write:
        src = os.path.join(ROOT, "monst3r-slam_amd", "csrc", "gemm_table.inc")
        lines = open(src).read().splitlines()
        keyre = re.compile(r"^\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+),")
        wins = {(r["M"], r["N"], r["K"], r["batch"], r["flags"], r["mode"]): r for r in rows
                if r["pp_us"] < (1 - args.min_gain) * r["base_us"]}
        out, seen = [], set()
        for ln in lines:
            mt = keyre.match(ln)
            k = tuple(int(v) for v in mt.groups()) if mt else None
            if k in wins:
                r = wins[k]
                ln = (f"{{{k[0]}, {k[1]}, {k[2]}, {k[3]}, {k[4]}, {k[5]}, {r['pp_cfg']}, 1, 0}},  "
                      f"// {r['base_us']:.1f} -> {r['pp_us']:.1f} us "
                      f"({'T256PP' if r['pp_cfg'] == 15 else 'T192PP'}, round 6)")
                seen.add(k)
            out.append(ln)
        for k, r in wins.items():
            if k not in seen:
                out.append(f"{{{k[0]}, {k[1]}, {k[2]}, {k[3]}, {k[4]}, {k[5]}, {r['pp_cfg']}, 1, "
                           f"0}},  // {r['base_us']:.1f} -> {r['pp_us']:.1f} us "
                           f"({'T256PP' if r['pp_cfg'] == 15 else 'T192PP'}, round 6)")
        path = os.path.join(os.path.dirname(args.out), "gemm_table_pp.inc")
        open(path, "w").write("\n".join(out) + "\n")
        print("wrote", path, len(wins), "classes to T256PP")


if __name__ == "__main__":
    main()
