#!/bin/bash
# the walk with the block's old rows in LDS (no wait on a fresh load inside
# a row), the pair split's side-stream window A/B in one process
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pairsplit.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "blocked_sweep or sequential or pair_split" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/seq_timing.py --only D,E,R --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seqprof.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/rank_shape_timing.py --shards 8,4 --layout pairs --side 0,1,0,1 --steps 10 > $OUT/rank_side.log 2>&1 || exit $?
echo ALL DONE
