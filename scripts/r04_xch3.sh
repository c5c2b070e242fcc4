#!/bin/bash
# Exchange-path staging A/B (FASTKMER_XCH_CUTS=0: stage every quarter, round 3; 1: at the job's cuts):
# one in-process rank at the configs[2] per-GPU load, two ranks at 3 GB each, alternated.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/xch3; mkdir -p $O
for v in 0 1 0 1; do
  FASTKMER_XCH_CUTS=$v timeout -k 10 300 python -u bench.py --rehearse-local 1 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl1_$v.json 2> $O/rl1_$v.err || { tail -5 $O/rl1_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rl1 c3 xch_cuts', sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/rl1_$v.json $v
done
for v in 0 1; do
  FASTKMER_XCH_CUTS=$v timeout -k 10 300 python -u bench.py --rehearse-local 2 --bytes-per-gpu 3000000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl2_$v.json 2> $O/rl2_$v.err || { tail -5 $O/rl2_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rl2 3g xch_cuts', sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/rl2_$v.json $v
done
