#!/bin/bash
# Round 6, 26th GPU call: does a 5-piece build (lib_p5, FK_STAGE_MAXP=5) cost configs[1] anything at its default
# 4 pieces (4 interleaved lines each), and the 5-piece cut set D at the configs[2] / configs[3] loads (2 each).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06z; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P5=FASTKMER_LIB=$R/fastkmer_amd/lib_p5/libfastkmer.so
D=FASTKMER_PIECE_CUTS=0.38,0.64,0.82,0.93
for r in 1 2 3 4; do
  line c2_p4_$r c2 X=1 || exit 1
  line c2_p5_$r c2 $P5 || exit 1
done
for r in 1 2; do
  line c3_p4_$r c3 X=1 || exit 1
  line c3_p5D_$r c3 $P5 $D || exit 1
  line c4_p4_$r c4 X=1 || exit 1
  line c4_p5D_$r c4 $P5 $D || exit 1
done
