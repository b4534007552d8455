#!/bin/bash
# round 5: one-pass logreg W image, ranking colcenter -- tests, S = 8 share, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13m
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_range.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_split.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "logreg or score or config_D" > $OUT/tests_logreg.log 2>&1 || exit $?
timeout -k 10 240 python3 scripts/rank_shape_timing.py --rest 0 --steps 10 --shards 8 --layout pairs --mode timer,plain > $OUT/s8.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
echo ALL DONE
