"""Summary of one replayed C3 step's launch timeline (bench.py --timeline-out): concurrency,
GEMM / attention busy time, idle gaps, and per-shape in-step durations.
  python tools/timeline_report.py gpurun_out/r03_timeline.json [> profiles/X.txt]"""
import collections
import json
import sys


def main(path):
    d = json.load(open(path))
    L = d["launches"]
    ev = []
    for x in L:
        kind = "gemm" if x["kind"] == "conv" else x["kind"]   # implicit-GEMM convs count as GEMM
        ev.append((x["start_us"], 1, kind))
        ev.append((x["end_us"], -1, kind))
    ev.sort()
    span = max(x["end_us"] for x in L) - min(x["start_us"] for x in L)
    conc = collections.Counter()
    busy = collections.Counter()
    active = collections.Counter()
    t_prev = ev[0][0]
    for t, dlt, k in ev:
        dt = t - t_prev
        n = sum(active.values())
        conc[min(n, 5)] += dt
        for kk in ("gemm", "attn"):
            if active[kk] > 0:
                busy[kk] += dt
        if n > 0:
            busy["any"] += dt
        active[k] += dlt
        t_prev = t
    print(f"step (HIP events) {d['step_ms']:.3f} ms; stamped span {span / 1e3:.3f} ms; "
          f"{len(L)} launches ({sum(1 for x in L if x['kind'] in ('gemm', 'conv'))} GEMM, "
          f"{sum(1 for x in L if x['kind'] == 'attn')} attention)")
    gf = sum(x["gflop"] for x in L if x["kind"] in ("gemm", "conv"))
    af = sum(x["gflop"] for x in L if x["kind"] == "attn")
    print(f"GEMM busy (union) {busy['gemm'] / 1e3:.3f} ms -> {gf / busy['gemm'] * 1e3:.0f} TF/s "
          f"({gf:.0f} GF); attention busy {busy['attn'] / 1e3:.3f} ms -> "
          f"{af / busy['attn'] * 1e3:.0f} TF/s; GEMM-or-attention {busy['any'] / 1e3:.3f} ms; "
          f"neither (other kernels / gaps) {(span - busy['any']) / 1e3:.3f} ms")
    print("concurrent GEMM/attention launches: " + ", ".join(
        f"{k}{'+' if k == 5 else ''}: {conc[k] / span * 100:.1f}%" for k in sorted(conc)))
    by = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for x in L:
        key = (x["kind"], tuple(x["dims"]))
        by[key][0] += 1
        by[key][1] += x["end_us"] - x["start_us"]
        by[key][2] += x["gflop"]
    print(f"\n{'kind':5s} {'dims (M,N,K,b | Sq,Sk,h,b)':28s} {'n':>4s} {'sum us':>9s} "
          f"{'avg us':>8s} {'TF/s':>7s}")
    for (k, dm), (n, us, g) in sorted(by.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{k:5s} {str(list(dm)):28s} {n:4d} {us:9.1f} {us / n:8.1f} {g / us * 1e3:7.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
