# validation of the shipped tree (smoke, GPU suite, bench, rocprof stats),
# then an in-box A/B of candidate-pass variants against it
set -o pipefail
TAG=r10c BSTEPS=20 STEPS="smoke tests bench prof" bash scripts/gpu_session.sh || exit 1
grep -q "tests exit 0" gpurun_out/r10c/steps.log || exit 1
L=dist-svgd_amd/dsvgd/_lib
MODE=rank SHARDS=1,8 TAG=r10c bash scripts/gpu_ab.sh $L/libdsvgd_hip_cand2.so $L/libdsvgd_hip_cb2048.so > gpurun_out/r10c/ab.txt 2>&1 || { tail -20 gpurun_out/r10c/ab.txt; exit 1; }
grep -E "lib=|shards" gpurun_out/r10c/ab_rank.log | cut -c1-300
