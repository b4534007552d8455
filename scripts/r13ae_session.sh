#!/bin/bash
# Gram A/B of the packed epilogue (dsvgd_gram_set_packed): timing, Gram tests, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13ae
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/gram_ab.py > $OUT/ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gram.py tests/test_gpu_parity.py -k "gram or median or bracket" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 scripts/gram_ab.py > $OUT/prof.log 2>&1 || exit $?
echo ALL DONE
