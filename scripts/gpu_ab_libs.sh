# phi_probe (distances + phi_mm at the headline shape) over the shipped
# library and the A/B builds named on the command line, one process each.
set -o pipefail
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
CFG=${CONFIGS:-h2:sym}
for L in "" "$@"; do
  echo "lib=${L:-shipped}" >> $OUT/ab.log
  timeout -k 10 180 python scripts/phi_probe.py --configs $CFG ${L:+--lib $L} >> $OUT/ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab.log
