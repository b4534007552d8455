#!/bin/bash
# phi_w1 DS 4 with 2 slices: parity, bench, rocprof stats, HBM traffic passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13p
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "symmetric or full_size or config_D_bench" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/symrow_ab.py --rounds 3 --steps 4 > $OUT/ab.log 2>&1 || exit $?
TAG=r13p STEPS="bench prof pmc pmcw" bash scripts/gpu_session.sh || exit $?
echo ALL DONE
