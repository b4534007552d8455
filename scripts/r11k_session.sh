#!/bin/bash
# the W2 eps divisor sweep, then the headline bench with its rocprof stats and
# the PMC fetch / write passes (profiles/latest_summary.json)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11k
mkdir -p $OUT
timeout -k 10 500 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 --theta 4,8,16,32 \
  > $OUT/w2_theta.log 2>&1 || exit $?
TAG=r11k STEPS="bench prof pmc pmcw" BSTEPS=20 bash scripts/gpu_session.sh || exit $?
echo ALL DONE
