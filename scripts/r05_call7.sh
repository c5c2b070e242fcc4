#!/bin/bash
# Round 5 seventh GPU call: the exchange in ten steps per job (one-rank configs[2] rehearsal + its tail
# timeline), the two-rank configs[1] rehearsal, the default bench line, useHT / configs[3] refresh.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05g; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_pieces.py \
  -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 5 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, d.get("buckets_rank0"))
PYEOF
}
run c3_rehearse1 X=1 python -u bench.py --rehearse-local 1 --workload c3 $B || exit 1
run c2_rehearse2 X=1 python -u bench.py --rehearse-local 2 $B || exit 1
run c2_rehearse1 X=1 python -u bench.py --rehearse-local 1 $B || exit 1
run c4_sorted X=1 python -u bench.py --workload c4 $B || exit 1
run c4_ht X=1 python -u bench.py --workload c4 --use-ht $B || exit 1
run c3_ht X=1 python -u bench.py --workload c3 --use-ht $B || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xch1 -o run -- python3 $R/bench.py --workload c3 \
  --rehearse-local 1 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_xch1.json 2> $O/prof_xch1.err || { echo "prof xch failed"; tail -20 $O/prof_xch1.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_xch1/run_kernel_trace.csv | tail -4
