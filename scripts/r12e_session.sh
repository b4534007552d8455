#!/bin/bash
# W2 cost tiles 128 x 128: W2 parity tests, the 8192 x 65536 timing, kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r12e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "w2" > gpurun_out/r12e/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/w2_timing.py --shapes 8192x65536x256,2048x16384x256 > gpurun_out/r12e/w2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r12e/prof -o run --output-format csv -- python3 scripts/w2_timing.py --shapes 8192x65536x256 > gpurun_out/r12e/prof.log 2>&1
rc=$?
tail -3 gpurun_out/r12e/tests.log; cat gpurun_out/r12e/w2.log
exit $rc
