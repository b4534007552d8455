#!/bin/bash
# round 5 first box: the new pair-split / RCCL-p2p / W2-stall tests, then the bench + rocprof
set -o pipefail
export TMPDIR=/tmp
TAG=r13a STEPS="pfab tests bench prof" BSTEPS=20 \
  PYTEST_K="pair_split or rccl_world1 or tail_stall or config_D_sharded or w2_assignment or w2_warm" \
  bash scripts/gpu_session.sh || exit $?
echo ALL DONE
