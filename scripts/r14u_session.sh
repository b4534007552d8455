#!/bin/bash
# round 6: rank shares at S = 1, 8 (row blocks and the pair split, the
# product defaults) on the final Gram
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14u
mkdir -p $OUT
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 1,8,4,2 --mode plain,timer --rest 0 --layout both > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/rank.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shards'], d['layout'], d['mode'], d.get('full_square'), d.get('t_splits'), round(d['ms_per_step_no_comm'],3), d['stages_ms'])"
echo ALL DONE
