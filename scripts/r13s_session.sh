#!/bin/bash
# XCD map for the batched forward partials (mask 4) at S = 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13s
mkdir -p $OUT
timeout -k 10 400 python3 scripts/rank_shape_timing.py --rest 0 --steps 10 --shards 8 --layout pairs --mode plain,timer --xmap 1,5,1,5 > $OUT/s8.log 2>&1 || exit $?
echo ALL DONE
