#!/bin/bash
# round 6 (session 2): gathered-data all_scores (the own block's scores over
# every rank's data, score blocks all-gathered): the distributed tests on
# gloo ranks sharing the GPU, the bench's 2-rank rehearsal, and one rank's
# S = 8 share with both score forms against S = 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16e
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_pairsplit.py tests/test_bench.py tests/test_gpu_split.py -m gpu -x -v --timeout 600 --timeout-method thread -k "sharded or pair_split or two_ranks or prior_weight" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python scripts/rank_shape_timing.py --shards 1,8 --layout both --mode plain --scores gathered,allreduce > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
timeout -k 10 600 python scripts/rank_shape_timing.py --shards 8 --layout pairs --mode timer --scores gathered,allreduce >> $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
grep "^{" $OUT/rank.log | cut -c1-400
echo ALL DONE
