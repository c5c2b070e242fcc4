#!/bin/bash
# GPU session: the -m gpu suite (without the 50 GB load test), then the
# configs[2] per-GPU-load test at a 10 GB rehearsal and at the full 50 GB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
tag=${1:-r02}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
FASTKMER_C3_GB=10 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 280 --timeout-method thread \
    -p no:cacheprovider -k per_gpu_load > $OUT/c3load10_$tag.log 2>&1
rc=$?; tail -3 $OUT/c3load10_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 380 --timeout-method thread \
    -p no:cacheprovider -k per_gpu_load > $OUT/c3load50_$tag.log 2>&1
rc=$?; tail -3 $OUT/c3load50_$tag.log; exit $rc
