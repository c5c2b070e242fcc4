#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ph in 0 1 2 3 99; do
  FASTKMER_COUNT_MODE=1 FASTKMER_DEBUG_PHASE=$ph timeout -k 10 120 python3 scripts/count_once.py > gpurun_out/pp_$ph.log 2>&1 || { cat gpurun_out/pp_$ph.log; exit 1; }
  echo "phase $ph: $(grep count gpurun_out/pp_$ph.log)"
done
