#!/bin/bash
# round 6 (session 3): full-size Gauss-Seidel parity with refreshed logreg
# scores (configs D and E) + the sweep tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r16i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 400 --timeout-method thread -k "refreshed or sweep" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -8 $OUT/tests.log
echo ALL DONE
