# final validation of the shipped tree: smoke, the GPU suite, bench, rocprof stats
set -o pipefail
TAG=r10e BSTEPS=20 STEPS="smoke tests bench prof" bash scripts/gpu_session.sh || exit 1
grep -q "tests exit 0" gpurun_out/r10e/steps.log
