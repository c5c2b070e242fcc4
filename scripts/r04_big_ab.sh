#!/bin/bash
# Big-tier table A/B at the configs[2] per-GPU load (N = 1): 6144 slots / 4096 distinct (60 KB, two
# workgroups per CU) against 5120 / 3072 (52 KB, three per CU; lib_big5120), alternated.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/bigab; mkdir -p $O
for v in base big5120 base big5120; do
  if [ $v = base ]; then unset FASTKMER_LIB; else export FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so; fi
  timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()}, d['buckets_rank0'])" $O/$v.json $v
done
unset FASTKMER_LIB
