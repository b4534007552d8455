#!/bin/bash
# the fused logreg score kernel: parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13v
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fused" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/gxd_ab.py --switch dsvgd_logreg_set_fused > $OUT/ab.log 2>&1 || exit $?
echo ALL DONE
