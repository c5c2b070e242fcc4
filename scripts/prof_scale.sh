#!/bin/bash
# kernel stats of rank 0's count at N-GPU weak scaling (scripts/probe_scale.py N)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; tag=${1:-sc}; N=${2:-8}
timeout -k 10 200 python3 -u scripts/probe_scale.py 1 || exit 1
timeout -k 10 200 python3 -u scripts/probe_scale.py 2 || exit 1
timeout -k 10 200 python3 -u scripts/probe_scale.py 4 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv \
  -- python3 -u $ROOT/scripts/probe_scale.py $N > $OUT/prof_$tag.log 2>&1
rc=$?; cat $OUT/prof_$tag.log | grep "N="; exit $rc
