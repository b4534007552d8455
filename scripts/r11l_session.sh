#!/bin/bash
# the whole GPU suite and the smoke test on the current tree
set -o pipefail
export TMPDIR=/tmp
TAG=r11l STEPS="smoke tests" bash scripts/gpu_session.sh || exit $?
grep -q "tests exit 0" gpurun_out/r11l/steps.log || exit 1
echo ALL DONE
