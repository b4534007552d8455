# phi_mm A/B of library builds against the shipped library: timing per D
# layout + every 256th phi row compared with the shipped kernel's.
#   CFGS=h2:sym,h2:full bash scripts/w1_ab.sh dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_w1a.so ...
set -o pipefail
OUT=gpurun_out/${TAG:-w1}; mkdir -p $OUT
CFGS=${CFGS:-h2:sym,h2:full}
timeout -k 10 200 python scripts/phi_probe.py --configs $CFGS --dump $OUT/ship > $OUT/probe_ship.log 2>&1 || exit 1
grep -v amdgpu $OUT/probe_ship.log
for L in "$@"; do
  n=$(basename $L .so)
  timeout -k 10 200 python scripts/phi_probe.py --configs $CFGS --lib $L --dump $OUT/$n > $OUT/probe_$n.log 2>&1 || exit 1
  grep -v amdgpu $OUT/probe_$n.log | sed "s/^/$n /"
  for c in ${CFGS//,/ }; do c=${c/:/_}; echo "  $c $(python scripts/dump_compare.py $OUT/ship_$c.npy $OUT/${n}_$c.npy)"; done
done
