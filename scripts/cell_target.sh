#!/bin/bash
# Count stage vs the cell target (FASTKMER_DEBUG_CELL_TARGET) at the configs[2] shape (1 GB, 3 Gbp
# virtual genome, B = 8192) and at configs[1]: gpurun_out/ct.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for wl in c3 c2; do
for ct in 0 192 128 96; do
  FASTKMER_DEBUG_CELL_TARGET=$ct timeout -k 10 200 python -u bench.py --workload $wl --bytes-per-gpu 1000000000 --steps 3 --warmup 1 --no-cpu-baseline > $O/ct.json 2>> $O/ct.err || exit 1
  python -c "import json; d=json.load(open('$O/ct.json')); print('$wl target $ct', round(d['ms_per_step'],2), round(d['device_resident_ms_per_step'],2), {k: round(v,2) for k,v in d['device_resident_stages_ms'].items()})" | tee -a $O/ct.log
done
done
