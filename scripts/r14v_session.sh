#!/bin/bash
# round 6: W2 cost store policy A/B; the pair split with the full square from
# S = 4 on (pair-split tests, sharded config D, rank shares S = 2, 4, 8)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14v
mkdir -p $OUT
timeout -k 10 300 python scripts/w2_cost_ab.py > $OUT/w2ab.log 2>&1 || { tail -20 $OUT/w2ab.log; exit 1; }
grep "^{" $OUT/w2ab.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_pairsplit.py tests/test_gpu_configs.py -m gpu -x -v -k "pair or sharded" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/rank_shape_timing.py --shards 2,8 --mode plain --rest 0 --layout pairs > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/rank.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shards'], d['layout'], d['mode'], d.get('full_square'), round(d['ms_per_step_no_comm'],3))"
echo ALL DONE
