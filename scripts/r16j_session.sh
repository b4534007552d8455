#!/bin/bash
# round 6 final tree: every BASELINE.json configuration (Jacobi, one GPU) and
# the reference-default sequential order at configs D and E
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16j
mkdir -p $OUT
timeout -k 10 400 python scripts/configs_bench.py > $OUT/configs.log 2>&1 || { tail -20 $OUT/configs.log; exit 1; }
grep "^{" $OUT/configs.log | cut -c1-300
timeout -k 10 500 python scripts/seq_timing.py --only D,E --rows-sample 0 > $OUT/seq.log 2>&1 || { tail -20 $OUT/seq.log; exit 1; }
grep "^{" $OUT/seq.log | cut -c1-400
echo ALL DONE
