#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r13e
timeout -k 10 200 python scripts/xstream_probe.py > gpurun_out/r13e/xs.log 2>&1 || exit $?
timeout -k 10 200 python scripts/pipe_debug.py 4096 > gpurun_out/r13e/dbg.log 2>&1 || exit $?
echo ALL DONE
