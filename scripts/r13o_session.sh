#!/bin/bash
# XCD slice map for DS 0 (window / row blocks) and DS 4: parity, A/B at S = 1 and S = 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13o
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pairsplit.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "symmetric or full_size or row_block or pair or config_D" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/symrow_ab.py --rounds 3 --steps 4 > $OUT/ab.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/rank_shape_timing.py --rest 0 --steps 10 --shards 8 --layout pairs --mode plain --xmap 1,0,1,0 > $OUT/s8.log 2>&1 || exit $?
echo ALL DONE
