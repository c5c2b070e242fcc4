#!/bin/bash
# Round-end measurement set on HEAD: whole -m gpu suite (configs[2] 50 GB load included),
# bench line (CPU baseline, host leg), useHT bench line, rocprof kernel stats of the bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-final}
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -rs > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 400 python3 bench.py > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
rc=$?; cut -c1-400 $OUT/bench_$tag.json; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python3 bench.py --use-ht --no-cpu-baseline --no-host-leg > $OUT/bench_ht_$tag.json 2> $OUT/bench_ht_$tag.err
rc=$?; cut -c1-300 $OUT/bench_ht_$tag.json; [[ $rc -ne 0 ]] && exit $rc
bash scripts/prof_bench.sh $tag --no-host-leg || exit 1
