#!/bin/bash
# round 6: is the pipelined sweep host-bound? (enqueue time vs sweep time),
# configs D and E (E with the pipeline forced on)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14y
mkdir -p $OUT
timeout -k 10 600 python scripts/seq_timing.py --only D --rows-sample 0 --reserve 0,8 --graphs 1 > $OUT/seqD.log 2>&1 || { tail -20 $OUT/seqD.log; exit 1; }
grep "^{" $OUT/seqD.log | cut -c1-500
timeout -k 10 600 python scripts/seq_timing.py --only E --rows-sample 0 --reserve 0,8 --pipe-max-d 1024 > $OUT/seqE.log 2>&1 || { tail -20 $OUT/seqE.log; exit 1; }
grep "sweep_ms_by_side_reserve" $OUT/seqE.log | cut -c1-500
echo ALL DONE
