#!/bin/bash
# round 6: split-role Gram probes (B ring depth, priority, epilogue cost) vs
# gram_w1 in-process, a PMC stall pass on the split-role Gram; then the W2
# session and the rank shares
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14e
mkdir -p $OUT
for v in 1 2 3 4 5; do
  timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on $v --off 0 > $OUT/ab_$v.log 2>&1 || { tail -20 $OUT/ab_$v.log; exit 1; }
  echo "variant $v: $(grep '^{' $OUT/ab_$v.log)"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $OUT/pmc -o run --output-format csv -- python3 scripts/gram_ab.py --switch dsvgd_gram_set_rs --on 1 --off 0 > $OUT/pmc.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 scripts/gram_ab.py --switch dsvgd_gram_set_rs --on 1 --off 0 > $OUT/pmc2.log 2>&1 || exit 1
echo PMC DONE
