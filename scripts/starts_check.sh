#!/bin/bash
# staged pieces with / without the per-bucket piece starts: pieces tests, then the bench step for both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/ps_tests.log 2>&1 || { tail -40 $O/ps_tests.log; exit 1; }
tail -2 $O/ps_tests.log
for st in 1 0 1 0; do
  FASTKMER_STAGED_STARTS=$st timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-device-leg > $O/ps.json 2>> $O/ps.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/ps.json')); print('starts $st', round(d['ms_per_step'],2), round(d['value']/1e9,2), {k: round(v,2) for k,v in d['stages_ms'].items()})" | tee -a $O/ps.log
done
