#!/bin/bash
# round 6: where the W2 warm solve's time goes at R = 1, 65536^2 (rocprofv3
# kernel stats over w2_timing's cost-only, cold and warm calls)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14r
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 > $OUT/w2prof.log 2>&1 || { tail -20 $OUT/w2prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r14r/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:90], r["Calls"], "%.3f ms avg" % (float(r["AverageNs"]) / 1e6), "%.1f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
echo ALL DONE
