"""Per-kernel averages of every counter in a rocprofv3 --pmc run directory.

    python scripts/pmc_table.py gpurun_out/<tag>/<step> [substring ...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    dur = collections.defaultdict(list)
    if tr:
        for r in csv.DictReader(open(tr[0])):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if keys and not any(s in k for s in keys):
            continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, c in per.items():
        n = len(disp[k])
        ms = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
        print("%s  [%d dispatches, %.3f ms]" % (k[:110], n, ms))
        wc = c.get("SQ_WAVE_CYCLES")
        for name, v in sorted(c.items()):
            extra = ""
            if wc and name.startswith("SQ_WAIT") or name == "SQ_ACTIVE_INST_ANY":
                extra = "  (%.1f%% of wave cycles)" % (100 * v / wc) if wc else ""
            print("    %-32s %14.4g%s" % (name, v / n, extra))


if __name__ == "__main__":
    main()
