#!/bin/bash
# round 6 final tree (session 3) measurement: bench (with the CPU baseline), rocprofv3
# kernel stats of the bench, PMC passes over the bench (MFMA busy, stalls,
# FETCH_SIZE, WRITE_SIZE) for profiles/latest_summary.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r16h}
mkdir -p $OUT
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep "^{" $OUT/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
P="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d $OUT/mfma -o run --output-format csv -- $P > $OUT/mfma.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $OUT/stall -o run --output-format csv -- $P > $OUT/stall.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $P > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $P > $OUT/write.log 2>&1 || exit 1
timeout -k 10 400 python scripts/rank_shape_timing.py --shards 1,8 --layout pairs --mode plain --scores gathered,allreduce > $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
timeout -k 10 300 python scripts/rank_shape_timing.py --shards 8 --layout pairs --mode timer --scores gathered,allreduce >> $OUT/rank.log 2>&1 || { tail -20 $OUT/rank.log; exit 1; }
grep "^{" $OUT/rank.log | cut -c1-300
echo ALL DONE
