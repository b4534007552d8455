#!/bin/bash
# concurrency check of the step's kernels; W2 R = 1 and R = 8 re-timed; the
# rank shares at S = 1 / 8 with the forward split-K; bench + rocprof
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13f
TAG=r13f STEPS="tests" PYTEST_K="side_stream_work" bash scripts/gpu_session.sh || exit $?
timeout -k 10 500 python scripts/w2_timing.py --shapes 65536x65536x256,8192x65536x256 \
  > gpurun_out/r13f/w2.log 2>&1 || exit $?
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 1,8 --rest 0 \
  > gpurun_out/r13f/rank.log 2>&1 || exit $?
TAG=r13f STEPS="bench prof" BSTEPS=20 bash scripts/gpu_session.sh || exit $?
echo ALL DONE
