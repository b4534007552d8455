export TMPDIR=/tmp
T=${T:-r2t}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/x3tests.log 2>&1 && \
AB_VARIANTS='{"x3":{}}' AB_SQ_VARIANTS='{"t128":{"DSVGD_GRAM_TILE":"128"},"t256":{}}' timeout -k 10 300 python scripts/ab_kernels.py > gpurun_out/$T/ab.log 2>&1 && \
AB_VARIANTS='{"x3":{}}' timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/pmc -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 > gpurun_out/$T/pmc.log 2>&1
echo rc=$?
tail -2 gpurun_out/$T/x3tests.log
grep -v amdgpu.ids gpurun_out/$T/ab.log | grep sqdist
