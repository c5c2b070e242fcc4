#!/bin/bash
# useHT at the configs[3] per-GPU load (6.25 GB, k = 55) and at configs[2]'s (6.25 GB, k = 28, B = 8192).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/htfull; mkdir -p $O
for wl in c4 c3; do
  FASTKMER_BENCH_MEMINFO=1 timeout -k 10 400 python -u bench.py --workload $wl --use-ht --steps 3 --warmup 1 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'useHT', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()}, d['distinct_rank0'])" $O/$wl.json $wl
  grep meminfo $O/$wl.err || true
done
