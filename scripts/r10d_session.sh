# the shipped tree (two-slot candidate passes, batched sample gathers): the
# select / bracket / Gram tests, rank-share A/B against the previous build,
# bench and rocprof stats
set -o pipefail
OUT=gpurun_out/r10d; mkdir -p $OUT
L=dist-svgd_amd/dsvgd/_lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "median or bracket or gram_w1 or config_D_bench or sample" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
MODE=rank SHARDS=1,8 TAG=r10d bash scripts/gpu_ab.sh $L/libdsvgd_hip_prev.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -E "lib=|shards" $OUT/ab_rank.log | cut -c1-300
TAG=r10d BSTEPS=20 STEPS="bench prof" bash scripts/gpu_session.sh
