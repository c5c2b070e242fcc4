#!/bin/bash
# Count-stage A/B: targeted parity tests, then bench (HBM-resident leg) per env variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-ws}; wl=${2:-c2}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "wave_tables or variants or random or two_word or grouped or c3_shape" \
    > $OUT/tests_$tag.log 2>&1
rc=$?; tail -3 $OUT/tests_$tag.log; [[ $rc -ne 0 ]] && exit $rc
i=0
for v in "FASTKMER_WAVE_SLOTS=768" "FASTKMER_WAVE_SLOTS=1024" "FASTKMER_WAVE_SLOTS=768" "FASTKMER_WAVE_SLOTS=1024"; do
  i=$((i+1))
  env $v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-host-leg --workload $wl > $OUT/bench_${tag}_$i.json 2> $OUT/bench_${tag}_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_${tag}_$i.json')); print('$v', round(d['value']/1e9,2), d['stages_ms'])"
done
bash scripts/prof_bench.sh $tag --no-host-leg --workload $wl || exit 1
