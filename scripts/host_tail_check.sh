#!/bin/bash
# Host-side tail of the staged host-input step: the piece / parity / comm GPU tests, the default
# bench line, then one bench run with FASTKMER_HOST_TRACE=1 (host timestamps of the partition and
# count steps on stderr: gpurun_out/ht_trace.err)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_parity.py tests/test_gpu_comm.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/ht_tests.log 2>&1 || { tail -40 $O/ht_tests.log; exit 1; }
tail -2 $O/ht_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ht_bench$i.json 2>> $O/ht_bench.err || exit 1
  python -c "import json; d=json.load(open('$O/ht_bench$i.json')); print(round(d['ms_per_step'],2), round(d['value']/1e9,2), 'dev', round(d['device_resident_ms_per_step'],2))"
done
FASTKMER_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/ht_trace.json 2> $O/ht_trace.err || exit 1
