#!/bin/bash
# wave-tier sort: GPU suite, then count kernels for the tier variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-sort}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
bash scripts/probe_tiers.sh $tag ${VARIANTS:--} > $OUT/tiers_$tag.txt 2>&1
rc=$?; grep -v simple_timer $OUT/tiers_$tag.txt; exit $rc
