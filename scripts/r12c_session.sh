#!/bin/bash
# the other BASELINE configurations at S = 1 on the final tree
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r12c
mkdir -p $OUT
timeout -k 10 600 python -u scripts/configs_bench.py > $OUT/configs.log 2>&1 || exit $?
echo ALL DONE
