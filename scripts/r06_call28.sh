#!/bin/bash
# Round 6, 28th GPU call (a re-run of the 27th's lines: that box's H2D ran at 123-127 ms): 5 staged pieces per job at most (FK_STAGE_MAXP=5), the 5-piece cuts for 64-bit jobs of
# >= 4 GB: the whole GPU suite, then A/B lines against lib_p4 (FK_STAGE_MAXP=4, round 6's 4-piece schedule)
# at configs[1] and the configs[2] / configs[3] loads, interleaved.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zb; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P4=FASTKMER_LIB=$R/fastkmer_amd/lib_p4/libfastkmer.so
for r in 1 2 3; do
  line c2_p5_$r c2 X=1 || exit 1
  line c2_p4_$r c2 $P4 || exit 1
done
for r in 1 2; do
  line c3_p5_$r c3 X=1 || exit 1
  line c3_p4_$r c3 $P4 || exit 1
done
line c4_p5 c4 X=1 || exit 1
line c4_p4 c4 $P4 || exit 1
