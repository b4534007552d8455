#!/bin/bash
# Gram bracket epilogue without the per-value diagonal select: in-box A/B
# (shipped = new, ab = old), then the median / Gram / config tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13h
for r in 1 2; do
  TAG=r13h MODE=probe CONFIGS=h2:sym bash scripts/gpu_ab.sh dist-svgd_amd/dsvgd/_lib/libdsvgd_hip_ab.so || exit $?
done
TAG=r13h STEPS="tests" PYTEST_K="median or gram or bracket" \
  bash scripts/gpu_session.sh || exit $?
echo ALL DONE
