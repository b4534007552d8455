# rank_shape_timing (S = $SHARDS) on the shipped library and on each A/B
# build named on the command line, one process each.
set -o pipefail
OUT=gpurun_out/${TAG:-rankab}; mkdir -p $OUT
for L in "" "$@"; do
  echo "lib=${L:-shipped}" >> $OUT/rank_ab.log
  timeout -k 10 300 python scripts/rank_shape_timing.py --shards ${SHARDS:-1,8} ${L:+--lib $L} >> $OUT/rank_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/rank_ab.log | cut -c1-330
