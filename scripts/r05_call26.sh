#!/bin/bash
# Round 5 26th GPU call: the exchange path's staging cuts at the configs[2] load (one in-process rank,
# FASTKMER_PIECE_CUTS), and 64 MB H2D segments for a 1 GB job (lib_seg16) against 32 MB.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05z; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, round(d.get("pcie_h2d_GBps") or 0, 2))
PYEOF
}
for rep in 1 2; do
  for cuts in 0.4,0.7,0.9 0.4,0.7,0.86 0.35,0.65,0.84 0.45,0.72,0.88; do
    run x1_$cuts FASTKMER_PIECE_CUTS=$cuts python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
  done
  run c2_default X=1 python -u bench.py $B || exit 1
  run c2_seg16 FASTKMER_LIB=$R/fastkmer_amd/lib_seg16/libfastkmer.so python -u bench.py $B || exit 1
done
