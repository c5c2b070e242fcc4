#!/bin/bash
# Host-input step vs piece cuts (FASTKMER_PIECE_CUTS): gpurun_out/cuts.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for cut in 0.5 0.55 0.6 0.65 0.7 "0.45,0.8" "0.5,0.85"; do
  FASTKMER_PIECE_CUTS=$cut timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-device-leg > $O/cut.json 2>> $O/cuts.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/cut.json')); print('cuts $cut', round(d['ms_per_step'],2), round(d['value']/1e9,2), {k: round(v,2) for k,v in d['stages_ms'].items()})" | tee -a $O/cuts.log
done
