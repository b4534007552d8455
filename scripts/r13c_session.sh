#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13c
timeout -k 10 300 python scripts/det_probe.py > gpurun_out/r13c/det.log 2>&1 || exit $?
echo ALL DONE
