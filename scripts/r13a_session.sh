#!/bin/bash
# round 5 first box: phi_w1 prefetch A/B, the S = 8 share with / without the
# forward split-K and prefetch, the new pair-split / RCCL-p2p / W2-stall
# tests, then the bench + rocprof
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13a
TAG=r13a STEPS="pfab" bash scripts/gpu_session.sh || exit $?
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 8 --layout pairs --fwdz 1,0 --pf 0,1 \
  > gpurun_out/r13a/rank.log 2>&1 || exit $?
TAG=r13a STEPS="tests bench prof" BSTEPS=20 \
  PYTEST_K="pair_split or rccl_world1 or tail_stall or config_D_sharded or w2_assignment or w2_warm" \
  bash scripts/gpu_session.sh || exit $?
echo ALL DONE
