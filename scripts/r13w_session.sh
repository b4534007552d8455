#!/bin/bash
# the fused logreg score as default: logreg / score / config tests, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13w
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "logreg or score or config_D or config_E or smoke or bench" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/gxd_ab.py --switch dsvgd_logreg_set_fused > $OUT/ab.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/rank_shape_timing.py --rest 0 --steps 10 --shards 1,8 --layout pairs --mode plain > $OUT/rank.log 2>&1 || exit $?
echo ALL DONE
