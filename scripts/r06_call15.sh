#!/bin/bash
# Round 6, 15th GPU call: staged-piece cut sets (FASTKMER_PIECE_CUTS; 5 pieces need lib_p5, FK_STAGE_MAXP=5)
# at the configs[2] / configs[3] loads and configs[1], one line each (screening).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06o; mkdir -p $O
cd $R
B="--steps 4 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P5=FASTKMER_LIB=$R/fastkmer_amd/lib_p5/libfastkmer.so
for wl in c3 c4 c2; do
  line ${wl}_def $wl X=1 || exit 1
  line ${wl}_A $wl FASTKMER_PIECE_CUTS=0.5,0.77,0.92 || exit 1
  line ${wl}_B $wl FASTKMER_PIECE_CUTS=0.45,0.72,0.9 || exit 1
  line ${wl}_C $wl $P5 FASTKMER_PIECE_CUTS=0.42,0.7,0.86,0.95 || exit 1
  line ${wl}_D $wl $P5 FASTKMER_PIECE_CUTS=0.38,0.64,0.82,0.93 || exit 1
done
