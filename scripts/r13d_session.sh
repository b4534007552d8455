#!/bin/bash
# the pipelined wide Gauss-Seidel sweep: parity tests, then config D / E / R
# sequential steps with and without the pipeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13d
TAG=r13d STEPS="tests" PYTEST_K="pipelined_wide or blocked_sweep or sequential_wide or config_C_sequential or sampler_blocked" \
  bash scripts/gpu_session.sh || exit $?
grep -q "tests exit 0" gpurun_out/r13d/steps.log || exit 1
timeout -k 10 500 python scripts/seq_timing.py --only D,R --pipeline 1,0 --rows-sample 0 \
  > gpurun_out/r13d/seq.log 2>&1 || exit $?
echo ALL DONE
