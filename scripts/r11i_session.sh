#!/bin/bash
# the W2 tail with one bidding wave (the others join only the scans), the
# walk's rm along the column loop and cheaper block end: parity, timings
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "w2 or wasserstein or blocked_sweep or sequential" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 --keep 0 > $OUT/w2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w2prof -o run --output-format csv -- \
  python3 scripts/w2_timing.py --shapes 8192x65536x256 --keep 0 > $OUT/w2prof.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/seq_timing.py --only D,E --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seqprof.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/walk_probe.py > $OUT/walk_probe.log 2>&1 || exit $?
echo ALL DONE
