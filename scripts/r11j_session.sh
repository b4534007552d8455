#!/bin/bash
# the walk's column loop over f32x4 column quads with the moved rows split
# over wave groups (dp % 256 == 0): parity, probe, the default-order timing
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r11j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v -x \
  --timeout 300 --timeout-method thread -k "blocked_sweep or sequential" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/walk_probe.py > $OUT/walk_probe.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/seq_timing.py --only D,E,R --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seqprof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seqprof.log 2>&1 || exit $?
echo ALL DONE
