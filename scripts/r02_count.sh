#!/bin/bash
# sorted-count changes: GPU suite, configs[2] rehearsal, rank-0 count at N = 1 and 8, bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-cnt}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
FASTKMER_C3_GB=10 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 280 --timeout-method thread \
    -p no:cacheprovider -k per_gpu_load > $OUT/c3load10_$tag.log 2>&1
rc=$?; grep "configs\[2\]\|passed\|failed" $OUT/c3load10_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 200 python3 -u scripts/probe_scale.py 1 || exit 1
timeout -k 10 200 python3 -u scripts/probe_scale.py 8 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-leg > $OUT/bench_$tag.log 2>&1
rc=$?; tail -1 $OUT/bench_$tag.log | cut -c1-300; exit $rc
