#!/bin/bash
# Submit one gpurun call, waiting while the pool reports no free box / slot
# (gpurun exit 3 or a "transient" status: nothing ran, nothing was charged).
# Any call that actually ran -- pass or fail -- ends the loop: a failing GPU
# step is never resubmitted.
#   scripts/gpurun_when_free.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then
    echo "gpurun rc=$rc (attempt $i)" >> "$out"
    exit $rc
  fi
  sleep 150
done
echo "gave up: pool busy" >> "$out"
exit 3
