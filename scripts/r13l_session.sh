#!/bin/bash
# launch gaps: the rank step with stage events / without / as one HIP graph;
# the one-wave window split (W_SPLITS=0) against the old rule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13l
mkdir -p $OUT
R="python3 scripts/rank_shape_timing.py --rest 0 --steps 10"
timeout -k 10 240 $R --shards 8 --layout pairs --mode timer,plain,graph --set W_SPLITS=8,0 > $OUT/s8.log 2>&1 || exit $?
timeout -k 10 240 $R --shards 4 --layout pairs --mode plain,graph --set W_SPLITS=4,0 > $OUT/s4.log 2>&1 || exit $?
timeout -k 10 240 $R --shards 1 --layout rows --mode timer,plain,graph > $OUT/s1.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
echo ALL DONE
