#!/bin/bash
# the one-wave Gauss-Seidel walk: parity tests, then config D / E / R
# sequential steps with the one-wave and the four-wave walk
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13d
TAG=r13d STEPS="tests" PYTEST_K="one_wave_walk or blocked_sweep or sequential_wide or config_C_sequential or sampler_blocked" \
  bash scripts/gpu_session.sh || exit $?
grep -q "tests exit 0" gpurun_out/r13d/steps.log || exit 1
timeout -k 10 600 python scripts/seq_timing.py --only D,R,E --walk 1,4 --rows-sample 0 \
  > gpurun_out/r13d/seq.log 2>&1 || exit $?
echo ALL DONE
