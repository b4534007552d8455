#!/bin/bash
# round 6 (session 2): the fused R = 1 warm start (violation + first-round
# scans in one pass): tests, A/B timing, kernel trace of the warm solve
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "w2" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for f in 1 0 1; do
  timeout -k 10 300 python scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 --fuse-first $f > $OUT/w2_fuse$f.log 2>&1 || { tail -20 $OUT/w2_fuse$f.log; exit 1; }
  grep -o '"warm_next_ms": [0-9.]*' $OUT/w2_fuse$f.log
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 scripts/w2_timing.py --shapes 65536x65536x256 --cost h2 > $OUT/w2prof.log 2>&1 || { tail -20 $OUT/w2prof.log; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/w2_trace_tail.py "$f" 60 > $OUT/tail.log
cat $OUT/tail.log
echo ALL DONE
