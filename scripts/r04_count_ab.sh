#!/bin/bash
# Count-stage layout A/B at configs[1] (HBM-resident leg of bench.py): the default two-level expansion
# (records -> super-cells -> cells of ~150 keys, wave tier) against one level straight into cells of
# ~1.5-2.6 K keys counted by the block / big tiers (no `mid` materialisation).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/count_ab; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('device_resident_stages_ms'), d.get('buckets_rank0'))" $O/$n.json $n
}
run base
run l1_1500 FASTKMER_EXPAND_LEVELS=1 FASTKMER_DEBUG_CELL_TARGET=1500
run l1_2600 FASTKMER_EXPAND_LEVELS=1 FASTKMER_DEBUG_CELL_TARGET=2600
run l1_800 FASTKMER_EXPAND_LEVELS=1 FASTKMER_DEBUG_CELL_TARGET=800
