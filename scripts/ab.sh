#!/bin/bash
# A/B timing of one env knob on the count stage: bash scripts/ab.sh VAR "v1 v2 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $2; do
  env "$1=$v" timeout -k 10 120 python3 scripts/count_once.py > gpurun_out/ab_$v.log 2>&1 || { cat gpurun_out/ab_$v.log; exit 1; }
  echo "$1=$v: $(grep count gpurun_out/ab_$v.log)"
done
