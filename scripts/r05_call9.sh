#!/bin/bash
# Round 5 ninth GPU call: staged piece cuts (FASTKMER_PIECE_CUTS) at configs[1] and the configs[2] load:
# the last piece is expanded after the last byte, so its share is the tail's; earlier pieces must finish
# while the later ones land (expansion ~7 ms per GB against 18 ms of H2D per GB).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05i; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()})
PYEOF
}
for cuts in 0.4,0.7,0.9 0.5,0.8,0.93 0.6,0.86,0.96 0.55,0.83,0.95 0.4,0.7,0.9; do
  run c2_$cuts FASTKMER_PIECE_CUTS=$cuts python -u bench.py $B || exit 1
  run c3_$cuts FASTKMER_PIECE_CUTS=$cuts python -u bench.py --workload c3 $B || exit 1
done
for v in rankown default rankown; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_$v $L python -u bench.py $B || exit 1
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
done
