#!/bin/bash
# useHT k <= 32: heavy groups in 8192-slot 64-bit tables (FASTKMER_HT_BIG64, auto by the distinct ratio).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/ht5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hash.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
probe() {  # name env...
  local n=$1; shift
  env "$@" FK_BYTES=999999906 timeout -k 10 300 python -u scripts/ht_probe.py 28 10 2048 100 > $O/probe_$n.txt 2>&1 || { tail -20 $O/probe_$n.txt; exit 1; }
  echo "== $n"; grep LDS $O/probe_$n.txt
}
probe off FASTKMER_HT_BIG64=0 || exit 1
probe auto FK_X=0 || exit 1
probe t2500 FASTKMER_HT_BIG64=2500 || exit 1
for v in 0 auto; do
  if [ $v = auto ]; then unset FASTKMER_HT_BIG64; else export FASTKMER_HT_BIG64=$v; fi
  timeout -k 10 300 python -u bench.py --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c1_ht_$v.json 2> $O/bench_c1_ht_$v.err || { tail -20 $O/bench_c1_ht_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c1 useHT big64', sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/bench_c1_ht_$v.json $v
done
