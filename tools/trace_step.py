"""Per-step kernel breakdown from a rocprofv3 kernel trace of bench.py: takes the last
tracking step (patchify .. track_finish) and sums device time per kernel family."""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/trace/bench_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "patchify_kernel" in r["Kernel_Name"]]
ends = [i for i, r in enumerate(rows) if "track_finish_kernel" in r["Kernel_Name"]]
e = ends[-1]
s = max(i for i in starts if i < e)
step = rows[s:e + 1]


def fam(n):
    m = re.search(r"gemm_kernel<([^>]*)>", n)
    if m:
        return "gemm<" + m.group(1) + ">"
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)
    return n[:60]


tot = collections.defaultdict(lambda: [0, 0])
busy = 0
for r in step:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy += d
    t = tot[fam(r["Kernel_Name"])]
    t[0] += 1
    t[1] += d
span = int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])
print(f"step span {span / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, launches {len(step)}")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{d / 1e6:8.3f} ms {100 * d / busy:5.1f}% n={n:4d} avg={d / n / 1e3:7.1f} us  {k}")
