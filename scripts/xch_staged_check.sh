#!/bin/bash
# staged pieces on the exchange path: comm + pieces tests, then 2-rank local rehearsals (staged / merge)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_pieces.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/xs_tests.log 2>&1 || { tail -40 $O/xs_tests.log; exit 1; }
tail -2 $O/xs_tests.log
for pm in 1 0; do
  FASTKMER_PIECE_MODE=$pm timeout -k 10 300 python -u bench.py --rehearse-local 2 --bytes-per-gpu 1000000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/xs.json 2>> $O/xs.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/xs.json')); print('local2 mode $pm', round(d['ms_per_step'],2), round(d['value']/1e9,2), {k: round(v,2) for k,v in d['stages_ms'].items()}, d['distinct_rank0'])" | tee -a $O/xs.log
done
