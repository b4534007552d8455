# Build an A/B variant of the library from a patched COPY of csrc/ (the
# product sources stay free of experiment switches):
#   bash scripts/ab_variant.sh NAME 'sed-expr' [file.hpp|file.hip ...]
# -> dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_NAME.so  (then scripts/gpu_ab.sh)
set -euo pipefail
NAME=$1; EXPR=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/dsvgd_ab/$NAME
rm -rf "$W"; mkdir -p "$W/csrc" "$W/build" /tmp/dsvgd_ab/include
cp "$ROOT"/include/dsvgd.h /tmp/dsvgd_ab/include/   # csrc includes ../../include/dsvgd.h
cp "$ROOT"/dist-svgd_amd/csrc/* "$W/csrc/"
for f in "$@"; do sed -i -e "$EXPR" "$W/csrc/$f"; done
for f in "$@"; do diff -q "$ROOT/dist-svgd_amd/csrc/$f" "$W/csrc/$f" > /dev/null && { echo "sed changed nothing in $f"; exit 1; }; done
for s in "$W"/csrc/*.hip; do
  b=$(basename "$s" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result \
    -c "$s" -o "$W/build/$b.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_$NAME.so" "$W"/build/*.o
echo "built dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_$NAME.so"
