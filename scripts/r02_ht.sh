#!/bin/bash
# useHT=1 bench line + kernel stats (extractKXmersHT path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; tag=${1:-ht}
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-leg --use-ht > $OUT/bench_$tag.log 2>&1
rc=$?; tail -1 $OUT/bench_$tag.log; [[ $rc -ne 0 ]] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv \
    -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-leg --use-ht > $OUT/prof_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
