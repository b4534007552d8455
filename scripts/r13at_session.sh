#!/bin/bash
# config E sweep kernels under rocprofv3 (the incremental walk at 4 columns per thread)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13at
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 scripts/seq_timing.py --only E --rows-sample 0 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
