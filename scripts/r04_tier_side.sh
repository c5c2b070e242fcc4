#!/bin/bash
# Block / big tiers on a side stream beside the wave tier (FASTKMER_TIER_SIDE=1) against one stream (0):
# count-variant parity tests, then configs[2] and configs[3] per-GPU loads and configs[1], alternated.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/tside; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_configs.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for wl in c3 c4 c2; do
  for v in 1 0 1 0; do
    FASTKMER_TIER_SIDE=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/${wl}_$v.json 2> $O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'tier_side', sys.argv[3], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/${wl}_$v.json $wl $v
  done
done
