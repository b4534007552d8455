#!/bin/bash
# the final tree's S = 8 pair-split rank step under rocprofv3 (kernel stats + trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13ac
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 scripts/rank_shape_timing.py --shards 8 --layout pairs --rest 0 --steps 5 --mode plain \
  > $OUT/rank.log 2>&1 || exit $?
echo ALL DONE
