#!/bin/bash
# the wide sweep's walk without in-loop global stores and its logreg score
# refresh, the pair split's window on a side stream: parity, then the default
# order's timing at config D / E, the rank shares and the kernel split
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pairsplit.py \
  -m gpu -v -x --timeout 300 --timeout-method thread \
  -k "blocked_sweep or sequential or pairsplit or pair_split or config_D_sharded or w2 or wasserstein" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rank_shape_timing.py --shards 4,8 --steps 5 > $OUT/rank.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seqprof.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/seq_timing.py --only D,E,R --rows-sample 1024 > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 --keep 1,0 > $OUT/w2.log 2>&1 || exit $?
echo ALL DONE
