#!/bin/bash
# XCD map with several column blocks (d = 1024): parity + config E A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13q
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread -k "symmetric or full_size or config_E or row_block" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 scripts/symrow_ab.py --rounds 2 --steps 2 --d 1024 > $OUT/ab_d1024.log 2>&1 || exit $?
echo ALL DONE
