export TMPDIR=/tmp
T=${T:-r1u}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/x3tests.log 2>&1 && \
AB_VARIANTS=${ABV:-'{"x3":{"ENGINE_X3":"1"},"f32":{"ENGINE_X3":"0"}}'} timeout -k 10 300 python scripts/ab_kernels.py > gpurun_out/$T/ab.log 2>&1 && \
AB_VARIANTS='{"x3":{"ENGINE_X3":"1"}}' timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/$T/pmcstall -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 > gpurun_out/$T/pmcstall.log 2>&1 && \
AB_VARIANTS='{"x3":{"ENGINE_X3":"1"}}' timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace -d gpurun_out/$T/pmcmfma -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 > gpurun_out/$T/pmcmfma.log 2>&1
echo rc=$?
tail -3 gpurun_out/$T/x3tests.log
grep -v amdgpu.ids gpurun_out/$T/ab.log | head -14
