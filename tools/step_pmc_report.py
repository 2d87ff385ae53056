"""Per-step summary of rocprofv3 runs of tools/step_prof.py (the bench's captured C3 step).

  python tools/step_pmc_report.py --pmc DIR [--trace DIR] [--flops-json F] --out profiles/X.json

--pmc DIR: a `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU GRBM_GUI_ACTIVE` run.
  SQ_VALU_MFMA_BUSY_CYCLES = 32 x the v_mfma_f32_32x32x16_bf16 instructions issued (16 per
  16x16x32; MI355X_MICROARCH.md 'Per-instruction cycle constants'), summed over the chip;
  GRBM_GUI_ACTIVE = GPU-busy cycles summed over the 8 XCDs.  Dispatches strictly between
  the two marker rownorm_kernel dispatches are the profiled steps.
--trace DIR: a `--kernel-trace --stats` run of the same script: per-kernel-class durations
  per step (traced: the tracer serialises the step's concurrent chains).
Derived per step: MFMA-busy SIMD-cycles by kernel class, the MFMA instructions they imply
(cycles / 32), the effective clock GRBM_GUI_ACTIVE / 8 / Σ dispatch time, and the MFMA
utilisation of the UNTRACED step = busy SIMD-cycles / (1024 SIMDs x clock x step time),
with the untraced step time taken from --step-ms (bench's ms_per_step)."""
import argparse
import collections
import csv
import glob
import json
import os


def _csv(d, suffix):
    f = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    if not f:
        raise SystemExit(f"no *{suffix} under {d}")
    return list(csv.DictReader(open(f[-1])))


def klass(name):
    if "gemm_kernel" in name or "splitk_reduce" in name:
        return "gemm"
    if "attn_kernel" in name or "attn_combine" in name:
        return "attn"
    return "other"


def between_markers(ids, names):
    m = [d for d in ids if "rownorm_kernel" in names[d]]
    if len(m) < 2:
        raise SystemExit("markers not found")
    return [d for d in ids if m[-2] < d < m[-1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--step-ms", type=float, required=True, help="untraced ms per step")
    ap.add_argument("--gemm-gflop", type=float, default=None,
                    help="algorithmic GEMM GFLOP per step (bench step_timeline)")
    ap.add_argument("--fetch", default=None, help="a --pmc FETCH_SIZE run of the same script")
    ap.add_argument("--write", default=None, help="a --pmc WRITE_SIZE run of the same script")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rows = _csv(a.pmc, "counter_collection.csv")
    ctr = collections.defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        ctr[d][r["Counter_Name"]] = ctr[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = between_markers(sorted(names), names)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in ids:
        k = klass(names[d])
        for c, v in ctr[d].items():
            per[k][c] += v
        per[k]["dispatches"] += 1
    S = a.steps
    out = {"steps": S, "dispatches_per_step": len(ids) / S, "by_class": {}}
    tot_busy = 0.0
    for k, v in per.items():
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / S
        tot_busy += busy
        out["by_class"][k] = {"dispatches": v["dispatches"] / S,
                              "mfma_busy_cycles": busy,
                              "mfma_32x32x16_equiv": busy / 32.0,
                              "implied_gflop": busy / 32.0 * 32768 / 1e9,
                              "sq_busy_cu": v.get("SQ_BUSY_CU", 0.0) / S,
                              "grbm_gui_active": v.get("GRBM_GUI_ACTIVE", 0.0) / S}
    out["mfma_busy_cycles_per_step"] = tot_busy
    if a.gemm_gflop:
        g = out["by_class"].get("gemm", {})
        out["gemm_counted_vs_algorithmic"] = g.get("implied_gflop", 0.0) / a.gemm_gflop
    if a.trace:
        tr = _csv(a.trace, "kernel_trace.csv")
        tn = {}
        dur = {}
        for r in tr:
            d = int(r["Dispatch_Id"])
            tn[d] = r["Kernel_Name"]
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # ms
        tids = between_markers(sorted(tn), tn)
        t0 = min(int(r["Start_Timestamp"]) for r in tr if int(r["Dispatch_Id"]) in set(tids))
        t1 = max(int(r["End_Timestamp"]) for r in tr if int(r["Dispatch_Id"]) in set(tids))
        cls = collections.defaultdict(float)
        for d in tids:
            cls[klass(tn[d])] += dur[d]
        byname = collections.defaultdict(lambda: [0, 0.0])
        for d in tids:
            byname[tn[d]][0] += 1
            byname[tn[d]][1] += dur[d]
        kern = sorted(({"name": n[:160], "per_step": c / S, "avg_us": t / c * 1e3,
                        "ms_per_step": t / S} for n, (c, t) in byname.items()),
                      key=lambda r: -r["ms_per_step"])
        out["traced"] = {"span_ms_per_step": (t1 - t0) * 1e-6 / S,
                         "kernel_ms_per_step": {k: v / S for k, v in cls.items()},
                         "dispatches_per_step": len(tids) / S, "kernels": kern}
    # HBM bytes per step and kernel class: FETCH_SIZE (KiB; x2 on gfx950 for 16-B-per-lane
    # reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (KiB), each from its own PMC run
    if a.fetch or a.write:
        hbm = collections.defaultdict(lambda: {"fetch_bytes": 0.0, "write_bytes": 0.0})
        for path, cname, key, scale in ((a.fetch, "FETCH_SIZE", "fetch_bytes", 2048.0),
                                        (a.write, "WRITE_SIZE", "write_bytes", 1024.0)):
            if not path:
                continue
            rr = _csv(path, "counter_collection.csv")
            nm, val = {}, collections.defaultdict(float)
            for r in rr:
                d = int(r["Dispatch_Id"])
                nm[d] = r["Kernel_Name"]
                if r["Counter_Name"] == cname:
                    val[d] += float(r["Counter_Value"])
            for d in between_markers(sorted(nm), nm):
                hbm[klass(nm[d])][key] += val[d] * scale / S
        for k in hbm:
            hbm[k]["bytes"] = hbm[k]["fetch_bytes"] + hbm[k]["write_bytes"]
        out["hbm"] = dict(hbm)
        out["hbm_bytes_per_step"] = sum(v["bytes"] for v in hbm.values())
    # GRBM_GUI_ACTIVE / 8 / traced kernel time reads above the 2.4 GHz maximum here (the
    # counter is not a plain per-XCD cycle count on this ROCm), so the utilisation is quoted
    # against the peak clock: a lower bound on the busy fraction at the clock actually held
    out["untraced_step_ms"] = a.step_ms
    out["mfma_util_step"] = tot_busy / (1024.0 * 2.4e9 * a.step_ms * 1e-3)
    out["note"] = ("MFMA utilisation = MFMA-busy SIMD-cycles per step (SQ_VALU_MFMA_BUSY_CYCLES, "
                   "PMC pass over the replayed step) / (1024 SIMDs x 2.4 GHz x untraced step "
                   "time): the share of the chip's peak MFMA cycles the step's MFMA "
                   "instructions occupy; the PMC run serialises dispatches, which does not "
                   "change the cycles the instructions take")
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
