#!/bin/bash
# round 6: kernel split of the pipelined config-D sweep (rocprofv3 stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14z
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seq.log 2>&1 || { tail -20 $OUT/seq.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r14z/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r["Name"][:80], r["Calls"], "%.1f us avg" % (float(r["AverageNs"]) / 1e3), "%.1f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
echo ALL DONE
