"""GEMM/attention launches of the last tracking step in a rocprofv3 kernel trace, grouped by
(kernel, grid): count, average and total device time."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/trace/bench_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "track_finish" in r["Kernel_Name"]]
starts = [i for i, r in enumerate(rows) if "patchify" in r["Kernel_Name"]]
e = ends[-1]
s = max(i for i in starts if i < e)
agg = collections.defaultdict(list)
for r in rows[s:e + 1]:
    n = r["Kernel_Name"]
    if "gemm_kernel" in n or "splitk" in n or "attn" in n or "layernorm" in n:
        tag = n.split("gemm_kernel")[-1][:28] if "gemm" in n else n[23:40]
        key = (tag, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"],
               r["Grid_Size_Z"])
        agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(k, len(v), "avg %.1f us" % (sum(v) / len(v) / 1e3), "tot %.3f ms" % (sum(v) / 1e6))
