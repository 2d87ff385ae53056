"""Report for tools/dec_trace.py traces: the last replay's launches grouped by (kernel,
grid), the sum of launch times, and the idle gaps between consecutive launches.
Usage: python tools/dec_trace_report.py DIR/..._kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last replay: from the last dec_embed-like first launch; replays are separated by the
# first copy_rows kernel of each decode
starts = [i for i, r in enumerate(rows) if "copy_rows" in r["Kernel_Name"]]
rep = rows[starts[-2] if len(starts) >= 2 else 0:]   # two copy_rows open each decode
agg = collections.defaultdict(list)
busy = 0
gaps = []
prev_end = None
for r in rep:
    n = r["Kernel_Name"]
    m = re.search(r"(gemm_kernel<[^>]*>|attn_kernel<[^>]*>|[a-z_0-9]+_kernel)", n)
    tag = m.group(1) if m else n[:40]
    blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * int(r["Grid_Size_Y"]) * \
        int(r["Grid_Size_Z"])
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    agg[(tag, blocks)].append(t1 - t0)
    busy += t1 - t0
    if prev_end is not None:
        gaps.append(t0 - prev_end)
    prev_end = t1
span = int(rep[-1]["End_Timestamp"]) - int(rep[0]["Start_Timestamp"])
print(f"launches {len(rep)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  "
      f"gaps {sum(gaps) / 1e3:.1f} us (median {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us)")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0][:60]:60s} blocks {k[1]:6d}  n {len(v):3d}  avg {sum(v) / len(v) / 1e3:7.2f} us  "
          f"tot {sum(v) / 1e3:8.1f} us")
