#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprof kernel stats.
# Stops at the first GPU fault / abort / timeout (exit 124,134,137,139 or >128).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name ($rc): stopping"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1500 python -u -m pytest ${TESTS:-tests} -m gpu -v -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} ;;
    bench) step bench 900 python bench.py --steps ${BSTEPS:-10} --warmup 3 ${BENCH_ARGS:-} ;;
    prof)  step prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    ab)    step ab 600 python scripts/ab_kernels.py ;;
    w2)    step w2 600 python scripts/w2_timing.py ${W2_ARGS:-} ;;
    diag)  step diag 600 python scripts/diag_precision.py ;;
    pmc)   step pmc 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmcclk) step pmcclk 900 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 --kernel-trace -d "$OUT/pmcclk" -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 ;;
    pmcstall) step pmcstall 900 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmcstall" -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 ;;
    pmcstallb) step pmcstallb 900 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmcstallb" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcmfma) step pmcmfma 900 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d "$OUT/pmcmfma" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcmfmaab) step pmcmfmaab 900 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace -d "$OUT/pmcmfmaab" -o run --output-format csv -- python3 scripts/ab_kernels.py --rounds 1 ;;
    configs) step configs 600 python scripts/configs_bench.py ;;
    notes) step notes 600 python scripts/notes_timing.py ;;
    pmcw)  step pmcw 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
  esac
done
echo ALL DONE
