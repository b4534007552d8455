#!/bin/bash
# kernel split of the S = 8 pair-split rank share (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13j
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13j/prof -o run --output-format csv -- \
  python3 scripts/rank_shape_timing.py --shards 8 --layout pairs --rest 0 --steps 5 \
  > gpurun_out/r13j/rank.log 2>&1 || exit $?
echo ALL DONE
