#!/bin/bash
# W2 tail: rescan floor from the cached columns and the bound column
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11z
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "w2 or wasserstein" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 > $OUT/w2.log 2>&1 || exit $?
echo ALL DONE
