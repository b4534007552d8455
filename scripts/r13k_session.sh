#!/bin/bash
# S = 8 pair split: sweep the split-K factors of the window, the row half,
# the antipodal partial and the forward batch (one rank's share, no comm)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13k
mkdir -p $OUT
R="python3 scripts/rank_shape_timing.py --shards 8 --layout pairs --rest 0 --steps 10"
timeout -k 10 200 $R --set W_SPLITS=0,4,16 > $OUT/w.log 2>&1 || exit $?
timeout -k 10 200 $R --set H_SPLITS=0,2,4,16 > $OUT/h.log 2>&1 || exit $?
timeout -k 10 200 $R --set REST_SPLITS=0,1,2,8 > $OUT/rest.log 2>&1 || exit $?
timeout -k 10 200 $R --fwdz 0,2,8 > $OUT/fwd.log 2>&1 || exit $?
echo ALL DONE
