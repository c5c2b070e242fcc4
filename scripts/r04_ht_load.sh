#!/bin/bash
# useHT group sizing (FASTKMER_HT_LOAD: expected distinct keys per group / table slots), configs[1] and
# the configs[2] shape at 1 GB (k = 28, B = 8192, 3 Gbp genome), alternated.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/htload; mkdir -p $O
for wl in c2 c3; do
  for v in 0.5 0.35 0.25 0.5 0.35 0.25; do
    FASTKMER_HT_LOAD=$v timeout -k 10 300 python -u bench.py --workload $wl --bytes-per-gpu 999999906 --use-ht --steps 5 --warmup 2 --no-cpu-baseline --no-device-leg > $O/${wl}_$v.json 2> $O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'load', sys.argv[3], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/${wl}_$v.json $wl $v
  done
done
