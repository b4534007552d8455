#!/bin/bash
# split-engine checks: tests/test_gpu_split.py, then the bench on h2 and x3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-h2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -m gpu -v -x --timeout 300 --timeout-method thread > "$OUT/split_tests.log" 2>&1
rc=$?; echo "split tests rc=$rc"; tail -3 "$OUT/split_tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for g in h2 x3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --gemm $g > "$OUT/bench_$g.log" 2>&1
  rc=$?; echo "bench $g rc=$rc"; tail -c 600 "$OUT/bench_$g.log"; echo
  [ $rc -eq 0 ] || exit $rc
done
