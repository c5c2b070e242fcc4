#!/bin/bash
# Round 6, 17th GPU call: cell width screening (FASTKMER_DEBUG_CELL_TARGET = average keys per cell of the largest
# bin: 256 default for 64-bit keys, 128 for 128-bit; one cell bit less per doubling) at the three loads.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06q; mkdir -p $O
cd $R
B="--steps 4 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d.get('buckets_rank0',{}); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()}, 'F', b.get('cell_bits'), 'buckets', b.get('all'), 'above', b.get('above_wave_tier'), b.get('kmers_above_wave_tier'))" $O/$name.json $name
}
line c3_def c3 X=1 || exit 1
line c3_t512 c3 FASTKMER_DEBUG_CELL_TARGET=512 || exit 1
line c3_t128 c3 FASTKMER_DEBUG_CELL_TARGET=128 || exit 1
line c4_def c4 X=1 || exit 1
line c4_t256 c4 FASTKMER_DEBUG_CELL_TARGET=256 || exit 1
line c4_t64 c4 FASTKMER_DEBUG_CELL_TARGET=64 || exit 1
line c2_def c2 X=1 || exit 1
line c2_t512 c2 FASTKMER_DEBUG_CELL_TARGET=512 || exit 1
line c2_t128 c2 FASTKMER_DEBUG_CELL_TARGET=128 || exit 1
