#!/bin/bash
# kernel-level A/B of two library builds on count_once.py (rocprof kernel stats per build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in old new; do
  if [ $v = old ]; then export FASTKMER_LIB=$GRAFT_REPO_ROOT/gpurun_ab/libfastkmer_old.so; else unset FASTKMER_LIB; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ab_$v$r -o run -- python3 $GRAFT_REPO_ROOT/scripts/count_once.py > $GRAFT_REPO_ROOT/$O/ab_$v$r.log 2>&1) || exit 1
  tail -1 $O/ab_$v$r.log
done
done
