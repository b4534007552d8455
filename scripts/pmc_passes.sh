# PMC passes over a probe command: one rocprofv3 --pmc run per counter group,
# each under its own limit (the hardware's per-block counter budget).
#   TAG=<dir under gpurun_out> PROBE="python3 scripts/phi_probe.py ..." bash scripts/pmc_passes.sh
set -o pipefail
OUT=gpurun_out/${TAG:-pmc}; mkdir -p $OUT
export TMPDIR=/tmp
P=${PROBE:-python3 scripts/phi_probe.py --configs h2:sym --reps 2}
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d $OUT/mfma -o run --output-format csv -- $P > $OUT/mfma.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $OUT/stall -o run --output-format csv -- $P > $OUT/stall.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $P > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $P > $OUT/write.log 2>&1 || exit 1
echo PMC DONE
