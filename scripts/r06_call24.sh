#!/bin/bash
# Round 6, 24th GPU call: staged piece cuts on the final tree (the last cut now beside the last expansion):
# 4-piece sets, and 5 pieces (lib_p5, FK_STAGE_MAXP=5), at the configs[2] / configs[3] loads; configs[1] with
# the default cuts on both builds (does a 5-piece build cost anything at 4 pieces?).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06x; mkdir -p $O
cd $R
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P5=FASTKMER_LIB=$R/fastkmer_amd/lib_p5/libfastkmer.so
for r in 1 2; do
  line c3_def$r c3 X=1 || exit 1
  line c3_A$r c3 FASTKMER_PIECE_CUTS=0.5,0.77,0.92 || exit 1
  line c3_D$r c3 $P5 FASTKMER_PIECE_CUTS=0.38,0.64,0.82,0.93 || exit 1
  line c3_E$r c3 $P5 FASTKMER_PIECE_CUTS=0.4,0.66,0.84,0.94 || exit 1
  line c2_def$r c2 X=1 || exit 1
  line c2_p5def$r c2 $P5 || exit 1
done
line c4_def c4 X=1 || exit 1
line c4_D c4 $P5 FASTKMER_PIECE_CUTS=0.38,0.64,0.82,0.93 || exit 1
line c4_E c4 $P5 FASTKMER_PIECE_CUTS=0.4,0.66,0.84,0.94 || exit 1
