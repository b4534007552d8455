# One GPU session: the -m gpu tests matching $1 (pytest -k), then optional
# timing scripts ($2: "probe", "rank", "bench" words).  Every step under its
# own time limit; the first failure ends the call.
set -o pipefail
K="$1"; WHAT="$2"; OUT=gpurun_out/${TAG:-chk}
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for w in $WHAT; do
  case $w in
    probe) timeout -k 10 240 python scripts/phi_probe.py --configs h2:sym,h2:full > $OUT/probe.log 2>&1 || exit 1; grep -v amdgpu.ids $OUT/probe.log ;;
    rank) timeout -k 10 300 python scripts/rank_shape_timing.py --shards ${SHARDS:-1,8} > $OUT/rank.log 2>&1 || exit 1; grep shards $OUT/rank.log ;;
    bench) timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1; tail -1 $OUT/bench.log | cut -c1-600 ;;
  esac
done
for w in $WHAT; do
  case $w in
    seq) timeout -k 10 600 python scripts/configs_bench.py --only ${SEQ:-B,C} --steps 1 --order sequential > $OUT/seq.log 2>&1 || exit 1; grep -v amdgpu.ids $OUT/seq.log ;;
  esac
done
