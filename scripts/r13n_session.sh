#!/bin/bash
# phi_w1 DS 4 (one launch per row on the symmetric layout): parity, A/B, profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13n
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "symmetric or full_size or row_block" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/symrow_ab.py --rounds 4 --steps 4 > $OUT/ab.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
echo ALL DONE
