# final check of the shipped tree: smoke, the select / bracket / Gram / config-D
# GPU tests, bench
set -o pipefail
TAG=r10e BSTEPS=20 STEPS="smoke tests bench" PYTEST_K="median or bracket or gram_w1 or config_D_bench or sample or smoke or phi_matches" bash scripts/gpu_session.sh || exit 1
grep -q "tests exit 0" gpurun_out/r10e/steps.log
