#!/bin/bash
# the antipodal partial beside the forward batch: pair-split parity, then the
# S = 8 / 4 shares with it on and off (twice, one process)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairsplit.py tests/test_gpu_configs.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "pair_split or config_D_sharded" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rank_shape_timing.py --shards 8 --layout pairs --rest 1,0,1,0 --steps 10 > $OUT/rank_rest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/rank_shape_timing.py --shards 1,2,4,8 --steps 10 > $OUT/rank.log 2>&1 || exit $?
echo ALL DONE
