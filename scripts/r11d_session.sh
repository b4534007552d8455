#!/bin/bash
# gram_w1 without the gate's spills (tests), rank shares with the sample
# shares filled, the sequential sweep's kernel split, bench + rocprof stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11d
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_pairsplit.py tests/test_gpu_configs.py \
  -m gpu -v -x --timeout 300 --timeout-method thread -k "gram or guard_fallback or all_scores_median or bench_step" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rank_shape_timing.py --steps 5 > $OUT/rank.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
echo ALL DONE
