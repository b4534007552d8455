#!/bin/bash
# final tree: smoke, the whole GPU suite, the headline bench and its rocprof stats
set -o pipefail
export TMPDIR=/tmp
TAG=r12f STEPS="smoke tests bench prof" BSTEPS=20 bash scripts/gpu_session.sh || exit $?
grep -q "tests exit 0" gpurun_out/r12f/steps.log || exit 1
echo ALL DONE
