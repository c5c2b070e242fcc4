#!/bin/bash
# Count-stage probes: bucket-kernel phases and scatter store cost (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for ph in 0 1 2 99; do
  FASTKMER_DEBUG_PHASE=$ph timeout -k 10 120 python3 scripts/count_once.py > $OUT/phase_$ph.log 2>&1 || exit 1
  echo "phase $ph: $(cat $OUT/phase_$ph.log)"
done
for sc in 0; do
  FASTKMER_DEBUG_SCATTER=$sc timeout -k 10 120 python3 scripts/count_once.py > $OUT/scatter_$sc.log 2>&1 || exit 1
  echo "scatter $sc: $(cat $OUT/scatter_$sc.log)"
done
