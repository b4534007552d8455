"""Summarise a gpu_session.sh run's rocprofv3 outputs into profiles/<tag>_*.

kernel_stats: per-kernel average duration (kernel-trace --stats);
hbm traffic: FETCH_SIZE / WRITE_SIZE per dispatch (separate --pmc passes),
reported in KiB by rocprofv3 -> bytes = value * 1024; FETCH_SIZE on gfx950
counts half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md section HBM), so fetch bytes are doubled.
    python scripts/pmc_summary.py gpurun_out/r1c r1
"""
import collections
import csv
import json
import os
import shutil
import sys


def mfma_pass(d, kernels):
    """MFMA utilisation per kernel from a pass of GRBM_GUI_ACTIVE,
    SQ_VALU_MFMA_BUSY_CYCLES and the SQ_INSTS_* counters
    (scripts/pmc_passes.sh "mfma"): GRBM_GUI_ACTIVE is summed over the 8
    XCDs, so the kernel's cycles are GRBM / 8 and the clock GRBM / 8 over
    its duration; MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES over those cycles x
    1024 SIMDs (256 CUs x 4)."""
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):
        return
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(path)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"]
    dur = {}
    tr = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(list)
    for disp, c in per.items():
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc <= 0 or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
            continue
        row = {"mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0)}
        if dur.get(disp, 0.0) > 1e-4:   # (short launches: the counters' window dominates)
            row["clock_ghz"] = cyc / dur[disp] / 1e9
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM",
                  "SQ_INSTS_VALU_MFMA_MOPS_F16"):
            if k in c:
                row[k.lower()] = c[k]
        agg[name[disp]].append(row)
    for k, rows in agg.items():
        dst = kernels.setdefault(k, {})
        for f in rows[0]:
            vals = [r[f] for r in rows if f in r]
            dst[f] = sum(vals) / len(vals)
        dst["mfma_pass_dispatches"] = len(rows)


def main(run, tag):
    os.makedirs("profiles", exist_ok=True)
    stats = os.path.join(run, "prof", "run_kernel_stats.csv")
    out = {"run": run, "kernels": {}}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join("profiles", "%s_kernel_stats.csv" % tag))
        for r in csv.DictReader(open(stats)):
            out["kernels"].setdefault(r["Name"], {})["avg_ms"] = float(r["AverageNs"]) / 1e6
            out["kernels"][r["Name"]]["calls"] = int(r["Calls"])
    for sub, cnt, corr in (("pmc", "FETCH_SIZE", 2.0), ("pmcw", "WRITE_SIZE", 1.0),
                           ("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        path = os.path.join(run, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == cnt:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0 * corr)
        for k, v in agg.items():
            key = "fetch_bytes_corrected" if cnt == "FETCH_SIZE" else "write_bytes"
            out["kernels"].setdefault(k, {})[key] = sum(v) / len(v)
    for sub in ("mfma", "pmcmfma"):
        mfma_pass(os.path.join(run, sub), out["kernels"])
    for k, v in out["kernels"].items():
        if "fetch_bytes_corrected" in v or "write_bytes" in v:
            v["hbm_bytes_per_launch"] = v.get("fetch_bytes_corrected", 0) + v.get("write_bytes", 0)
    with open(os.path.join("profiles", "%s_summary.json" % tag), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    if any("hbm_bytes_per_launch" in v for v in out["kernels"].values()):
        shutil.copy(os.path.join("profiles", "%s_summary.json" % tag),
                    os.path.join("profiles", "latest_summary.json"))
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("avg_ms", 0)):
        print("%-70s %8.3f ms  %s" % (k[:70], v.get("avg_ms", float("nan")),
              "%.2f GB" % (v["hbm_bytes_per_launch"] / 1e9) if "hbm_bytes_per_launch" in v else ""))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
