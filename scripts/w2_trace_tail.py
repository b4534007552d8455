"""Print the last N kernel launches of a rocprofv3 kernel trace (name, ms),
e.g. the warm W2 solve at the end of scripts/w2_timing.py.
    python scripts/w2_trace_tail.py <trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
t0 = int(rows[-n]["Start_Timestamp"])
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.3f ms  %8.3f ms  %s" % ((s - t0) / 1e6, (e - s) / 1e6, r["Kernel_Name"][:100]))
