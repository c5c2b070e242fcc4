#!/bin/bash
# Round 6, 18th GPU call: cell width for 64-bit keys (lib_t512: FK_CELL_TARGET64=512, one cell bit less than the
# default 256 at these loads), three lines each at the configs[2] load and configs[1], alternating.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06r; mkdir -p $O
cd $R
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d.get('buckets_rank0',{}); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()}, 'F', b.get('cell_bits'))" $O/$name.json $name
}
T=FASTKMER_LIB=$R/fastkmer_amd/lib_t512/libfastkmer.so
for r in 1 2 3; do
  line c3_def$r c3 X=1 || exit 1
  line c3_t512_$r c3 $T || exit 1
  line c2_def$r c2 X=1 || exit 1
  line c2_t512_$r c2 $T || exit 1
done
