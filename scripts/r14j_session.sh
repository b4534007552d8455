#!/bin/bash
# round 6: split-role Gram probes (E-only rate, E at priority 1) and the pair
# split with the diagonal square as one rectangle on the split-role Gram
# (FULL_SQUARE default on): pair-split and sharded config D tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14j
mkdir -p $OUT
for v in 6 7 1; do
  timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on $v --off 0 > $OUT/ab_$v.log 2>&1 || { tail -20 $OUT/ab_$v.log; exit 1; }
  echo "variant $v: $(grep '^{' $OUT/ab_$v.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairsplit.py tests/test_gpu_configs.py -m gpu -x -v -k "pair or sharded" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
echo ALL DONE
