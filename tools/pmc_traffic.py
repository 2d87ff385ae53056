"""HBM traffic of one pair inference's GEMM launches from rocprofv3 PMC passes
(tools/gpu_cmd_r1z.sh): FETCH_SIZE and WRITE_SIZE in separate passes, KiB units; on gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md
§HBM), so reads are doubled.  The last eager pair inference of the run is used (the
bench's serial roofline probe: patchify_kernel .. the head.2 conv with the fused DPT tail,
gemm_kernel<..., 517, ...> = BIAS|RELU|DPT_OUT; run the bench with --no-c5 --no-graph).
Writes profiles/<out>.json: per-launch and per-pair GEMM bytes, plus the L2 hit rate.
Usage: python tools/pmc_traffic.py gpurun_out/prof profiles/r01_pmc_gemm_traffic.json"""
import collections
import csv
import json
import sys


def load(path, counters):
    rows = list(csv.DictReader(open(path)))
    by = collections.defaultdict(dict)
    meta = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        if r["Counter_Name"] in counters:
            by[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = r["Kernel_Name"]
    return by, meta


def last_pair(meta):
    ids = sorted(meta)
    starts = [d for d in ids if "patchify_kernel" in meta[d]]
    ends = [d for d in ids if "gemm_kernel" in meta[d] and ", 517," in meta[d]]
    s = starts[-1]                       # the eager pair of the roofline replay recording
    e = min(d for d in ends if d > s)    # (its GEMM-only replay graph follows)
    return [d for d in ids if s <= d <= e]


root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_pmc_gemm_traffic.json"
fetch, mf = load(f"{root}/pmc_fetch/pmc_counter_collection.csv", {"FETCH_SIZE"})
write, mw = load(f"{root}/pmc_write/pmc_counter_collection.csv", {"WRITE_SIZE"})
hit, mh = load(f"{root}/pmc_hit/pmc_counter_collection.csv", {"TCC_HIT_sum", "TCC_MISS_sum"})
pf, pw, ph = last_pair(mf), last_pair(mw), last_pair(mh)
assert len(pf) == len(pw) == len(ph), (len(pf), len(pw), len(ph))
gemm = {"launches": 0, "read_bytes": 0.0, "write_bytes": 0.0, "tcc_hit": 0.0, "tcc_miss": 0.0}
allk = {"read_bytes": 0.0, "write_bytes": 0.0}
for a, b, c in zip(pf, pw, ph):
    name = mf[a]
    rd = 2.0 * fetch[a].get("FETCH_SIZE", 0.0) * 1024
    wr = write[b].get("WRITE_SIZE", 0.0) * 1024
    allk["read_bytes"] += rd
    allk["write_bytes"] += wr
    if "gemm_kernel" in name or "splitk_reduce" in name:
        gemm["launches"] += "gemm_kernel" in name
        gemm["read_bytes"] += rd
        gemm["write_bytes"] += wr
        gemm["tcc_hit"] += hit[c].get("TCC_HIT_sum", 0.0)
        gemm["tcc_miss"] += hit[c].get("TCC_MISS_sum", 0.0)
gemm["hbm_bytes_per_pair"] = gemm["read_bytes"] + gemm["write_bytes"]
gemm["hbm_bytes_per_launch"] = gemm["hbm_bytes_per_pair"] / max(1, gemm["launches"])
gemm["l2_hit_rate"] = gemm["tcc_hit"] / max(1.0, gemm["tcc_hit"] + gemm["tcc_miss"])
res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum, separate "
                 "passes; FETCH doubled (gfx950 wide-load correction); one eager pair inference",
       "gemm": gemm, "all_kernels_per_pair": allk, "kernels_in_pair": len(pf)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
