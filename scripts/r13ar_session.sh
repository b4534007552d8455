#!/bin/bash
# wide passes of about 128 rows (G = 128 // B): sweep parity, config D and E timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13ar
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "incremental_walk or blocked_sweep or sequential or gauss_seidel" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "wide_full_sweep or sequential" > $OUT/tests_full.log 2>&1 || exit $?
timeout -k 10 600 python3 -u scripts/seq_timing.py --only D,E --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
