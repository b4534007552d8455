#!/bin/bash
# the group correction with its loads issued ahead: parity, config D timing, sweep kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13al
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "wide_full_sweep" > $OUT/tests_full.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "incremental_walk or blocked_sweep" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only D --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
