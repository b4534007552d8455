#!/bin/bash
# round 6: pipelined sweep, the previous group's correction in one launch;
# forced-overlap and sweep tests, config D pipelined vs serial, group 1 vs 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r15b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v -k "forced_overlap or full_sweep or blocked_sweep" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python scripts/seq_timing.py --only D --rows-sample 0 --pipe 1,0 --group 1,2 > $OUT/seq.log 2>&1 || { tail -20 $OUT/seq.log; exit 1; }
grep "^{" $OUT/seq.log | cut -c1-400
echo ALL DONE
