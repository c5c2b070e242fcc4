#!/bin/bash
# Round 5 16th GPU call: the split's passes with 8 keys per lane in flight -- heavy-split parity,
# configs[1] / configs[2] load, kernel stats of configs[2].
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05p; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_heavy_bucket_split_vs_oracle" tests/test_gpu_hash.py \
  tests/test_gpu_pieces.py -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()})
PYEOF
}
run c2 X=1 python -u bench.py $B || exit 1
run c3 X=1 python -u bench.py --workload c3 $B || exit 1
run c2_b X=1 python -u bench.py $B || exit 1
run c3_b X=1 python -u bench.py --workload c3 $B || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 14
