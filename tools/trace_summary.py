"""Per-step kernel breakdown of the TIMED C3 sequence loop from a rocprofv3 kernel trace of
bench.py (rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- python bench.py).

The timed region is the last `steps` frames: from the end of the (steps+1)-th-last
seq_advance_kernel to the end of the last one (one advance per frame closes each step).
Per kernel family: launches and device time per step; GEMM time per step and the in-step
GEMM throughput against the pair's algorithmic GEMM flops (bench line
roofline.gemm_gflop_per_pair).  Kernels of all streams are summed (busy time can exceed the
span when the encoder prefetch overlaps the tracking chain).

  python tools/trace_summary.py DIR/run_kernel_trace.csv STEPS GFLOP_PER_STEP > out.txt"""
import collections
import json
import re
import sys


def fam(n):
    m = re.search(r"gemm_kernel<([^>]*)>", n)
    if m:
        return "gemm<" + m.group(1) + ">"
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


def main():
    path, steps, gflop = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    import csv
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adv = [i for i, r in enumerate(rows) if "seq_advance_kernel" in r[2]]
    assert len(adv) > steps, (len(adv), steps)
    t0 = rows[adv[-steps - 1]][1]
    t1 = rows[adv[-1]][1]
    reg = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, n in reg:
        t = tot[fam(n)]
        t[0] += 1
        t[1] += e - s
    span_ms = (t1 - t0) / 1e6 / steps
    busy_ms = sum(v[1] for v in tot.values()) / 1e6 / steps
    gemm_ms = sum(v[1] for k, v in tot.items() if k.startswith("gemm<") or "splitk" in k) / 1e6 / steps
    out = {"steps": steps, "ms_per_step_traced": span_ms, "kernel_busy_ms_per_step": busy_ms,
           "launches_per_step": len(reg) / steps, "gemm_ms_per_step": gemm_ms,
           "gemm_gflop_per_step": gflop,
           "gemm_tflops_in_step": gflop / gemm_ms if gemm_ms else None,
           "gemm_frac_of_2500": gflop / gemm_ms / 2500.0 if gemm_ms else None}
    print(json.dumps(out))
    for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{d / 1e6 / steps:8.4f} ms/step {100 * d / 1e6 / steps / busy_ms:5.1f}% "
              f"n/step={n / steps:6.2f} avg={d / n / 1e3:8.2f} us  {k}")


if __name__ == "__main__":
    main()
