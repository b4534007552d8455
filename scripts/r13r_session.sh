#!/bin/bash
# logreg G . Xd on phi_w1_kernel<0, 2, false>: tests, A/B, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13r
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "logreg or score or split" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/gxd_ab.py > $OUT/ab.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
echo ALL DONE
