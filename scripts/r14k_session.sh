#!/bin/bash
# round 6: W2 near-pair recompute lane-parallel (tests + 65536^2 timing); the
# split-role Gram's walk group 16 vs 8 (A/B, then PMC passes over both:
# MFMA busy, stalls, FETCH_SIZE, WRITE_SIZE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gram.py -m gpu -x -v -k "w2 or gram_rs" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 > $OUT/w2.log 2>&1 || { tail -20 $OUT/w2.log; exit 1; }
grep "^{" $OUT/w2.log | cut -c1-300
timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_group --on 16 --off 8 > $OUT/ab_group.log 2>&1 || { tail -20 $OUT/ab_group.log; exit 1; }
echo "group: $(grep '^{' $OUT/ab_group.log)"
TAG=r14k/pmc PROBE="python3 scripts/gram_ab.py --switch dsvgd_gram_set_group --on 16 --off 8" bash scripts/pmc_passes.sh || exit 1
echo ALL DONE
