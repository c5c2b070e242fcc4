#!/bin/bash
# Whole -m gpu suite (fused tests first), the phase probe, a bench line without the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-all}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/fused_$tag.log 2>&1
rc=$?; tail -3 $OUT/fused_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties --ignore tests/test_gpu_fused.py > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
bash scripts/fused_probe.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$tag.log 2>&1
rc=$?; tail -1 $OUT/bench_$tag.log; exit $rc
