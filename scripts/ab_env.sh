#!/bin/bash
# A/B of one environment knob on the host-input bench step: ab_env.sh VAR "v1 v2 ..." [tests...]
# (the tests run first, once, with the defaults; BENCH_ARGS: extra bench.py arguments)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
VAR=$1; VALS=$2; shift 2
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > $O/ab_tests.log 2>&1 || { tail -40 $O/ab_tests.log; exit 1; }
  tail -2 $O/ab_tests.log
fi
for v in $VALS $VALS; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $O/ab.json 2>> $O/ab.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/ab.json')); print('$VAR=$v', round(d['ms_per_step'],2), round(d['value']/1e9,2), 'dev', round(d['device_resident_ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" | tee -a $O/ab.log
done
