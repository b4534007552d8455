#!/bin/bash
# fused score: the sigma-hidden variant (2) against the shipped form (1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r13aa
mkdir -p $OUT
timeout -k 10 300 python3 scripts/gxd_ab.py --switch dsvgd_logreg_set_fused --on 2 --off 1 > $OUT/ab.log 2>&1 || exit $?
echo ALL DONE
