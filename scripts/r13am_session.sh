#!/bin/bash
# config D sweep by the wide pass's split-K slice count (0 = chosen, 256)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13am
mkdir -p $OUT
timeout -k 10 600 python3 -u scripts/seq_timing.py --only D --rows-sample 0 --splits 0,128,64,512 > $OUT/seq.log 2>&1 || exit $?
echo ALL DONE
