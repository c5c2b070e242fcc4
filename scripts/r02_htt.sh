#!/bin/bash
# useHT GPU tests first, then the whole -m gpu suite, then the HT bench + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-htt}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "ht or HT or hash" > $OUT/httests_$tag.log 2>&1
rc=$?; tail -3 $OUT/httests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
bash scripts/r02_ht.sh $tag
