"""Per-dispatch PMC values of a rocprofv3 --pmc run (tools only): the last N dispatches whose
kernel name contains a pattern, with the counter in MB (FETCH_SIZE doubled: gfx950 wide-load
correction, MI355X_MICROARCH.md §HBM).
  python tools/pmc_dispatches.py DIR COUNTER PATTERN [N]"""
import csv
import glob
import os
import sys

root, counter, pat = sys.argv[1:4]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
f = sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))[-1]
rows = {}
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] != counter or pat not in r["Kernel_Name"]:
        continue
    d = int(r["Dispatch_Id"])
    rows.setdefault(d, [r["Kernel_Name"], 0.0, r.get("Grid_Size", "")])
    rows[d][1] += float(r["Counter_Value"])
scale = (2048.0 if counter == "FETCH_SIZE" else 1024.0) / 1e6
for d in sorted(rows)[-n:]:
    name, v, grid = rows[d]
    i = name.find("<")
    print(d, name[i:i + 60], grid, f"{v * scale:.1f} MB")
