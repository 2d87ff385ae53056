"""Per-queue view of one tracking step from a rocprofv3 kernel trace of bench.py: the
step's span, each hardware queue's busy time, the main (tracking) queue's idle gaps, and
a run-length timeline of the main queue's kernel families (where its time goes)."""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/trace/bench_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "track_finish_kernel" in r["Kernel_Name"]]
e1, e0 = ends[-1], ends[-2]
step = rows[e0 + 1:e1 + 1]
main_q = rows[e1]["Queue_Id"]
t0 = int(rows[e0]["End_Timestamp"])
t1 = int(rows[e1]["End_Timestamp"])


def fam(n):
    m = re.search(r"gemm_kernel<([^>]*)>", n)
    if m:
        p = m.group(1).split(",")
        return "gemm" + ("_conv" if p[7].strip() != "0" else "") + f"<{p[0].strip()}x{p[1].strip()}>e{p[9].strip()}"
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)
    return n[:40]


busy = collections.defaultdict(int)
for r in step:
    busy[r["Queue_Id"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print(f"step span {(t1 - t0) / 1e3:.1f} us (track_finish to track_finish), kernels {len(step)}")
for q, b in busy.items():
    n = sum(1 for r in step if r["Queue_Id"] == q)
    print(f"  queue {q}{' (main)' if q == main_q else ''}: busy {b / 1e3:8.1f} us, {n} kernels")
mk = [r for r in step if r["Queue_Id"] == main_q]
gap, prev = 0, t0
for r in mk:
    s = int(r["Start_Timestamp"])
    gap += max(0, s - prev)
    prev = max(prev, int(r["End_Timestamp"]))
print(f"  main queue idle between its kernels: {gap / 1e3:.1f} us")
print("main-queue timeline (runs of one kernel family: count, busy us, span us):")
run = None
for r in mk + [None]:
    f = fam(r["Kernel_Name"]) if r else None
    if run and f == run[0]:
        run[1] += 1
        run[2] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        run[4] = int(r["End_Timestamp"])
        continue
    if run:
        print(f"  {(run[3] - t0) / 1e3:8.1f} {run[0]:44s} x{run[1]:3d} busy {run[2] / 1e3:7.1f} "
              f"span {(run[4] - run[3]) / 1e3:7.1f}")
    if r:
        run = [f, 1, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Start_Timestamp"]),
               int(r["End_Timestamp"])]
tot = collections.defaultdict(lambda: [0, 0])
for r in mk:
    t = tot[fam(r["Kernel_Name"])]
    t[0] += 1
    t[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print("main-queue totals by family:")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"  {d / 1e3:8.1f} us n={n:4d}  {k}")
