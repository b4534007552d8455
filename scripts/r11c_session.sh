#!/bin/bash
# Round-4 first GPU session: the new paths' parity (pair split, the wide
# Gauss-Seidel sweep, the guard fixes, config E end to end), then their
# timing (rank shares in both layouts, the default order at config D / E,
# the W2 auction), then the bench and its rocprof stats.  Stops at the first
# GPU fault / timeout (gpu_session.sh).
set -o pipefail
export TMPDIR=/tmp
TAG=r11c STEPS="tests" TESTS="tests/test_gpu_pairsplit.py tests/test_gpu_range.py" \
  bash scripts/gpu_session.sh || exit 1
grep -q "tests exit 0" gpurun_out/r11c/steps.log || exit 1
OUT=gpurun_out/r11c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v -x \
  --timeout 400 --timeout-method thread -k "blocked_sweep or sequential_wide or config_D_sharded or config_E_end or w2 or wasserstein" \
  > $OUT/tests2.log 2>&1; rc=$?; tail -3 $OUT/tests2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rank_shape_timing.py --steps 5 > $OUT/rank.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/seq_timing.py > $OUT/seq.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/w2_timing.py --shapes 2048x16384x256,8192x65536x256 > $OUT/w2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
echo ALL DONE
