#!/bin/bash
# Host-input step vs staged piece cuts / one-level small pieces: gpurun_out/sweep.log
# usage: staged_sweep.sh "CUTS:ONELEVEL" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for cfg in "$@"; do
  cut=${cfg%%:*}; ol=${cfg##*:}
  FASTKMER_PIECE_CUTS=$cut FASTKMER_STAGED_ONE_LEVEL=$ol timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-device-leg > $O/sw.json 2>> $O/sweep.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/sw.json')); print('cuts $cut one_level $ol', round(d['ms_per_step'],2), round(d['value']/1e9,2), {k: round(v,2) for k,v in d['stages_ms'].items()})" | tee -a $O/sweep.log
done
