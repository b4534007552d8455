#!/bin/bash
# round 6: W2 warm-start violation, eight rows per block (prices loaded once per
# chunk for eight rows): W2 tests, timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "w2" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python scripts/w2_timing.py --shapes 65536x65536x256,8192x65536x256 --cost h2 > $OUT/w2.log 2>&1 || { tail -20 $OUT/w2.log; exit 1; }
grep "^{" $OUT/w2.log | cut -c1-420
echo ALL DONE
