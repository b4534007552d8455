#!/bin/bash
# round 6: the split-role Gram -- gram tests (rs vs w1 bit-identical), the
# in-process A/B timing at the headline, then the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r14b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python scripts/gram_ab.py --switch dsvgd_gram_set_rs --on 1 --off 0 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -2 $OUT/ab.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 -c "
import json;l=[x for x in open('$OUT/bench.log') if x.startswith('{')][0];d=json.loads(l);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['stages_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
head -6 $OUT/prof/run_kernel_stats.csv | cut -c1-150
echo ALL DONE
