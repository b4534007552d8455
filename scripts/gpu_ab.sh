# In-box A/B of library builds (make -C dist-svgd_amd ab AB_FLAGS=...): one
# timing script over the shipped library and over each build named on the
# command line, one process per library (same box, back to back).
#   MODE=probe  scripts/phi_probe.py     (phi_mm + distances; CONFIGS=h2:sym,...)
#   MODE=rank   scripts/rank_shape_timing.py (stages of one rank's share; SHARDS=1,8)
#   MODE=cfg    scripts/configs_bench.py (BASELINE configs; CFGS=C)
#     bash scripts/gpu_ab.sh dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_x.so ...
set -o pipefail
MODE=${MODE:-probe}
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for L in "" "$@"; do
  echo "lib=${L:-shipped}" >> $OUT/ab_$MODE.log
  case $MODE in
    probe) timeout -k 10 180 python scripts/phi_probe.py --configs ${CONFIGS:-h2:sym} ${L:+--lib $L} ;;
    rank)  timeout -k 10 300 python scripts/rank_shape_timing.py --shards ${SHARDS:-1,8} ${L:+--lib $L} ;;
    cfg)   timeout -k 10 300 python scripts/configs_bench.py --only ${CFGS:-C} ${L:+--lib $L} ;;
  esac >> $OUT/ab_$MODE.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab_$MODE.log | cut -c1-400
