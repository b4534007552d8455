#!/bin/bash
# round 6: W2 cost (r14c), rank shares (r14d), pipelined sweep (r14g).
# A plain test failure (rc 1) moves on to the next session; a time limit,
# abort or fault (rc 124/134/137/139 or any other) ends the call there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in r14c r14d r14g; do
  bash scripts/${s}_session.sh
  rc=$?
  echo "== $s rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
