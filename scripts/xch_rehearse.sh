#!/bin/bash
# 2-rank local rehearsals of the configs[2] shape (staged / merge pieces) at BYTES per rank
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
B=${1:-3000000000}
for pm in 1 0 1 0; do
  FASTKMER_PIECE_MODE=$pm timeout -k 10 400 python -u bench.py --rehearse-local 2 --bytes-per-gpu $B --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/xr.json 2>> $O/xr.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/xr.json')); print('local2 bytes $B mode $pm', round(d['ms_per_step'],2), round(d['value']/1e9,2), {k: round(v,2) for k,v in d['stages_ms'].items()}, d['exchange']['steps'])" | tee -a $O/xr.log
done
