#!/bin/bash
# round 6: split-role Gram with the candidate stage in the read hand-off chunks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 1 5; do
  timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on $v --off 0 > $OUT/ab_$v.log 2>&1 || { tail -20 $OUT/ab_$v.log; exit 1; }
  echo "variant $v: $(grep '^{' $OUT/ab_$v.log)"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep "^{" $OUT/bench.log | cut -c1-300
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 1,8 --mode plain,timer --square 0,1 --rest 0 --layout both > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/rank.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shards'], d['layout'], d['mode'], d.get('full_square'), d.get('t_splits'), round(d['ms_per_step_no_comm'],3), d['stages_ms'])"
echo ALL DONE
