#!/bin/bash
# Round 6, 35th GPU call: configs[1] piece cuts -- a smaller last piece (expanded after the last byte) with
# five pieces; lib_mp128 lets a piece hold >= 64 MB (FK_MIN_PIECE_MB=128; the product: >= 128 MB).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zk; mkdir -p $O
cd $R
B="--steps 10 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
MP=FASTKMER_LIB=$R/fastkmer_amd/lib_mp128/libfastkmer.so
for r in 1 2 3; do
  line c2_def_$r c2 X=1 || exit 1
  line c2_A_$r c2 FASTKMER_PIECE_CUTS=0.4,0.6,0.75,0.9 || exit 1
  line c2_B_$r c2 $MP FASTKMER_PIECE_CUTS=0.4,0.65,0.85,0.95 || exit 1
  line c2_C_$r c2 $MP FASTKMER_PIECE_CUTS=0.42,0.7,0.88,0.96 || exit 1
  line c2_D_$r c2 $MP FASTKMER_PIECE_CUTS=0.5,0.8,0.93 || exit 1
  line c2_E_$r c2 $MP FASTKMER_PIECE_CUTS=0.45,0.75,0.92 || exit 1
done
