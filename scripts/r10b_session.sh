set -o pipefail
OUT=gpurun_out/r10b; mkdir -p $OUT
L=dist-svgd_amd/dsvgd/_lib
MODE=rank SHARDS=1,8 TAG=r10b bash scripts/gpu_ab.sh $L/libdsvgd_hip_candpf.so $L/libdsvgd_hip_candagg.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -E "lib=|shards" $OUT/ab_rank.log | cut -c1-330
for v in candpf candagg; do
  cp $L/libdsvgd_hip_$v.so $L/libdsvgd_hip.so
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "median or bracket or gram_w1 or config_D_bench" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
