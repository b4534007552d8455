#!/bin/bash
# W2 kernel trace of the final tail (cold, cold-next, warm solves)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r12b
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w2prof -o run --output-format csv -- \
  python3 scripts/w2_timing.py --shapes 8192x65536x256 > $OUT/w2prof.log 2>&1 || exit $?
echo ALL DONE
