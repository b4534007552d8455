# phi_mm A/B of phi_w1 builds against the shipped library (full D layout):
# timing + every 256th phi row compared with the shipped kernel's.
#   bash scripts/w1_ab.sh dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_w1a.so ...
set -o pipefail
OUT=gpurun_out/${TAG:-w1}; mkdir -p $OUT
timeout -k 10 200 python scripts/phi_probe.py --configs ${SHIPCFG:-h2:full} --dump $OUT/ship > $OUT/probe_ship.log 2>&1 || exit 1
grep -v amdgpu $OUT/probe_ship.log
for L in "$@"; do
  n=$(basename $L .so)
  timeout -k 10 200 python scripts/phi_probe.py --configs h2:full --lib $L --dump $OUT/$n > $OUT/probe_$n.log 2>&1 || exit 1
  echo "$n $(grep -v amdgpu $OUT/probe_$n.log) $(python scripts/dump_compare.py $OUT/ship_h2_full.npy $OUT/${n}_h2_full.npy)"
done
