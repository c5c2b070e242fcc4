#!/bin/bash
# Partition A/B at B = 8192 (configs[2] shape): parity tests, then the bench with the sorted record
# scatter for up to 8192 parts (FASTKMER_PART_SORTED=1) and the unsorted one above 2048 (=2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-part}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fused.py -m gpu -x -v \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "random or c3_shape or grouped or golden or many_bins" \
    > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
i=0
for v in 1 2 1 2; do
  i=$((i+1))
  FASTKMER_PART_SORTED=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-host-leg --workload c3 \
      > $OUT/bench_${tag}_$i.json 2> $OUT/bench_${tag}_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_${tag}_$i.json')); print('sorted=$v', round(d['value']/1e9,2), d['stages_ms'])"
done
bash scripts/prof_bench.sh $tag --no-host-leg --workload c3 || exit 1
