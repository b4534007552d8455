# configs_bench.py (configs $CFGS) on the shipped library and on each A/B
# build named on the command line, one process each.
set -o pipefail
OUT=gpurun_out/${TAG:-cfgab}; mkdir -p $OUT
for L in "" "$@"; do
  echo "lib=${L:-shipped}" >> $OUT/cfg_ab.log
  timeout -k 10 300 python scripts/configs_bench.py --only ${CFGS:-C} ${L:+--lib $L} >> $OUT/cfg_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/cfg_ab.log | cut -c1-400
