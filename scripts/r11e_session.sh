#!/bin/bash
# the wide sweep's faster reduce / walk barriers / thin-block Gram walk, the
# W2 phase tail: their tests, then timings
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11e
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gram.py tests/test_gpu_pairsplit.py \
  tests/test_gpu_configs.py -m gpu -v -x --timeout 300 --timeout-method thread \
  -k "blocked_sweep or sequential_wide or gram or w2 or wasserstein or all_scores_median or config_D_sharded" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seqprof.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/seq_timing.py > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 > $OUT/w2.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/rank_shape_timing.py --steps 5 > $OUT/rank.log 2>&1 || exit $?
echo ALL DONE
