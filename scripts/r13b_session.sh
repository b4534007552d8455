#!/bin/bash
# phi_w1 timing probes (DS 2) + determinism; the S = 8 share without the
# antipodal beside (the default) with / without the forward split-K; the W2
# stall test after the fix
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13b
timeout -k 10 300 python scripts/phi_pf_ab.py --forms 0,1,11,12,13,14,15 --rounds 3 \
  > gpurun_out/r13b/probe.log 2>&1 || exit $?
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 8 --layout pairs --rest 0 --fwdz 1,0 \
  > gpurun_out/r13b/rank.log 2>&1 || exit $?
TAG=r13b STEPS="tests" PYTEST_K="tail_stall or w2_assignment or w2_warm or w2_grad" \
  bash scripts/gpu_session.sh || exit $?
echo ALL DONE
