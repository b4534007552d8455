#!/bin/bash
# round 6: the W2 cost on the split-role MFMA Gram -- W2 tests, then the
# timing of both cost forms at R = 1 (65536 x 65536) and R = 8 (8192 x 65536)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "w2" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python scripts/w2_timing.py --shapes 65536x65536x256,8192x65536x256 --cost h2,exact > $OUT/w2.log 2>&1 || { tail -20 $OUT/w2.log; exit 1; }
cat $OUT/w2.log | grep "^{" | cut -c1-400
echo ALL DONE
