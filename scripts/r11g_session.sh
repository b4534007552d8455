#!/bin/bash
# the W2 auction's kernel split at m = 8192, n = 65536 (cold and warm), and
# the guard trip rate on converging runs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11g
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w2prof -o run --output-format csv -- \
  python3 scripts/w2_timing.py --shapes 8192x65536x256 --trace > $OUT/w2prof.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/guard_trip_rate.py --steps 300 > $OUT/guard.log 2>&1 || exit $?
echo ALL DONE
