#!/bin/bash
# round 6 (session 2): W2 cost line stores without spills (A/B, C identical),
# W2 tests, the prior-weighted logreg score test, the warm solve
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16d
mkdir -p $OUT
timeout -k 10 300 python scripts/w2_cost_ab.py --switch lines > $OUT/ab_lines.log 2>&1 || { tail -20 $OUT/ab_lines.log; exit 1; }
tail -1 $OUT/ab_lines.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -m gpu -x -v --timeout 300 --timeout-method thread -k "w2 or prior_weight or logreg_scores_fused" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 > $OUT/w2.log 2>&1 || { tail -20 $OUT/w2.log; exit 1; }
grep -o '"cost_ms": [0-9.]*\|"warm_next_ms": [0-9.]*\|"ms": [0-9.]*' $OUT/w2.log
echo ALL DONE
