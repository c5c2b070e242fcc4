#!/bin/bash
# fused map change: fused-kernel tests, whole GPU suite, map kernel timing at 512 threads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-map2}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties > $OUT/tests_$tag.log 2>&1
rc=$?; tail -2 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
FK_MAP_REPS=21 timeout -k 10 120 python3 scripts/map_once.py
