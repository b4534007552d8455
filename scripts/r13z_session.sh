#!/bin/bash
# the S = 1 / S = 8 rank shares on one box (plain, no stage markers) + the S = 1 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13z
mkdir -p $OUT
timeout -k 10 400 python3 scripts/rank_shape_timing.py --rest 0 --steps 10 --shards 1,2,4,8 --layout both --mode plain,timer > $OUT/rank.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
echo ALL DONE
