export TMPDIR=/tmp
T=${T:-r2x}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread -k logreg > gpurun_out/$T/x3tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k logreg > gpurun_out/$T/partests.log 2>&1 && \
AB_VARIANTS='{"x3":{}}' timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 2 > gpurun_out/$T/prof.log 2>&1 && \
DSVGD_LOGREG_Z=tile AB_VARIANTS='{"x3":{}}' timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof2 -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 2 > gpurun_out/$T/prof2.log 2>&1
echo rc=$?
tail -1 gpurun_out/$T/x3tests.log; tail -1 gpurun_out/$T/partests.log
grep -h logreg_z gpurun_out/$T/prof/run_kernel_stats.csv gpurun_out/$T/prof2/run_kernel_stats.csv | cut -c1-60,160-230
