#!/bin/bash
# GPU session: fused-kernel + streamed-ingest tests first (new code), then the
# whole -m gpu suite, a bench line and a rocprofv3 kernel-stats pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
tag=${1:-r02}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/fused_$tag.log 2>&1
rc=$?; tail -3 $OUT/fused_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$tag.log 2>&1
rc=$?; tail -1 $OUT/bench_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_configs.py::test_c3_per_gpu_load_rank0_properties --ignore tests/test_gpu_fused.py > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv \
    -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
