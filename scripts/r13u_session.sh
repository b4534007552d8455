#!/bin/bash
# grouped wide Gauss-Seidel sweep: parity, then config D timing by group
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13u
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sweep or sequential or blocked or gauss" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 scripts/seq_timing.py --only D --rows-sample 0 --group 1,2,4 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
