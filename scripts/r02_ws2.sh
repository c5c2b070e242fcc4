#!/bin/bash
# Count-stage check: targeted parity tests, then the bench (HBM-resident leg) at configs[1] and the
# configs[2] shape, and a kernel profile of configs[1].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-ws}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "wave_tables or variants or random or skewed or big_bins or c1 or c3_shape or golden" \
    > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
i=0
for wl in c2 c3 c2 c3; do
  i=$((i+1))
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-host-leg --workload $wl > $OUT/bench_${tag}_$i.json 2> $OUT/bench_${tag}_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_${tag}_$i.json')); print('$wl', round(d['value']/1e9,2), d['stages_ms'])"
done
bash scripts/prof_bench.sh $tag --no-host-leg || exit 1
