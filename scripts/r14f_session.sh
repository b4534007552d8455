#!/bin/bash
# round 6: the split-role Gram with the epilogue waves reading one slice
# ahead (compile-time slices, column data in registers, next tile's data
# loaded early): bit-identity tests, in-process A/B vs gram_w1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 1 5; do
  timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on $v --off 0 > $OUT/ab_$v.log 2>&1 || { tail -20 $OUT/ab_$v.log; exit 1; }
  echo "variant $v: $(grep '^{' $OUT/ab_$v.log)"
done
echo ALL DONE
