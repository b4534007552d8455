#!/bin/bash
# the round-5 tree: smoke, the whole GPU suite, the headline bench + rocprof
set -o pipefail
export TMPDIR=/tmp
TAG=r13i STEPS="smoke tests bench prof" BSTEPS=20 bash scripts/gpu_session.sh || exit $?
grep -q "tests exit 0" gpurun_out/r13i/steps.log || exit 1
echo ALL DONE
