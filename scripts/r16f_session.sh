#!/bin/bash
# round 6 (session 2): (1) W2 cost line stores without spills (A/B, C
# identical), W2 tests, the warm solve; (2) gathered-data all_scores (the own
# block's scores over every rank's data, prior x S, score blocks
# all-gathered; the fused score split over data slices for few particles):
# score tests, distributed tests on gloo ranks sharing the GPU, the bench's
# 2-rank rehearsal, one rank's S = 8 share with both score forms vs S = 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16f
mkdir -p $OUT
timeout -k 10 300 python scripts/w2_cost_ab.py --switch lines > $OUT/ab_lines.log 2>&1 || { tail -20 $OUT/ab_lines.log; exit 1; }
tail -1 $OUT/ab_lines.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -m gpu -x -v --timeout 300 --timeout-method thread -k "w2 or prior_weight or logreg_scores" > $OUT/tests_w2_scores.log 2>&1 || { tail -30 $OUT/tests_w2_scores.log; exit 1; }
tail -2 $OUT/tests_w2_scores.log
timeout -k 10 300 python scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 > $OUT/w2.log 2>&1 || { tail -20 $OUT/w2.log; exit 1; }
grep -o '"cost_ms": [0-9.]*\|"warm_next_ms": [0-9.]*\|"ms": [0-9.]*' $OUT/w2.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_pairsplit.py tests/test_bench.py -m gpu -x -v --timeout 600 --timeout-method thread -k "sharded or pair_split or two_ranks" > $OUT/tests_dist.log 2>&1 || { tail -40 $OUT/tests_dist.log; exit 1; }
tail -2 $OUT/tests_dist.log
timeout -k 10 600 python scripts/rank_shape_timing.py --shards 1,8 --layout both --mode plain --scores gathered,allreduce > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
timeout -k 10 600 python scripts/rank_shape_timing.py --shards 8 --layout pairs --mode timer --scores gathered,allreduce >> $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
grep "^{" $OUT/rank.log | cut -c1-420
echo ALL DONE
