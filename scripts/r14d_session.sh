#!/bin/bash
# round 6: one rank's share of the bench step at S = 1, 2, 4, 8 on one box
# (compute only), the pair split with the diagonal square on the 8-wave
# mirror kernel vs as one full rectangle on the split-role Gram
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14d
mkdir -p $OUT
timeout -k 10 600 python scripts/rank_shape_timing.py --shards 1,2,4,8 --mode plain,timer --square 0,1 --layout both > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/rank.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shards'], d['layout'], d['mode'], d.get('full_square'), round(d['ms_per_step_no_comm'],3), d['stages_ms'])"
echo ALL DONE
