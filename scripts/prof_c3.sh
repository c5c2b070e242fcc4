#!/bin/bash
# kernel stats of the configs[2] per-GPU-load test (rehearsal size FASTKMER_C3_GB, default 10)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; tag=${1:-c3}
export FASTKMER_C3_GB=${FASTKMER_C3_GB:-10}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv \
  -- python3 -u -m pytest $ROOT/tests/test_gpu_configs.py -x -q -s -p no:cacheprovider -k per_gpu_load > $OUT/prof_$tag.log 2>&1
rc=$?; grep "configs\[2\]" $OUT/prof_$tag.log; exit $rc
