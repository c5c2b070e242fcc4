#!/bin/bash
# Fused map iteration: fused-kernel tests vs the oracle, then the phase probe at 512 and 256 threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-map}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/fused_$tag.log 2>&1
rc=$?; tail -5 $OUT/fused_$tag.log; [[ $rc -ne 0 ]] && exit $rc
bash scripts/fused_probe.sh || exit 1
echo "--- 256 threads"; FASTKMER_FUSED_NT=256 FK_MAP_REPS=15 timeout -k 10 120 python3 scripts/map_once.py
