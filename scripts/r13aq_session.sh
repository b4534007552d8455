#!/bin/bash
# config E sweep by group size (blocks per wide pass; 16-row blocks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13aq
mkdir -p $OUT
timeout -k 10 700 python3 -u scripts/seq_timing.py --only E --rows-sample 0 --group 8,16 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
