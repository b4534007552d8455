#!/bin/bash
# round 6: split-role Gram: previous slot closed after slice 0, walk advanced after slice 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_parity.py -m gpu -x -v -k "gram or median or w2_cost_h2 or w2_h2" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on 1 --off 0 > $OUT/ab_1.log 2>&1 || { tail -20 $OUT/ab_1.log; exit 1; }
echo "rs vs w1: $(grep '^{' $OUT/ab_1.log)"
timeout -k 10 120 python scripts/gram_stamps.py > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
grep "^{" $OUT/stamps.log
echo ALL DONE
