#!/bin/bash
# Bench lines at 1 GB per GPU for the configs[2] / [3] / [4] shapes (c3, c4, c5): gpurun_out/shapes.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for wl in ${WLS:-c3 c4 c5}; do
  timeout -k 10 300 python -u bench.py --workload $wl --bytes-per-gpu 1000000000 --steps 5 --warmup 1 --no-cpu-baseline > $O/shape_$wl.json 2>> $O/shapes.err || exit 1
  python -c "import json; d=json.load(open('$O/shape_$wl.json')); print('$wl', round(d['value']/1e9,2), round(d['ms_per_step'],2), round(d['device_resident_value']/1e9,2), round(d['device_resident_ms_per_step'],2), {k: round(v,2) for k,v in d['device_resident_stages_ms'].items()})" | tee -a $O/shapes.log
done
