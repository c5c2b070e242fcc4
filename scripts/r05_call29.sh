#!/bin/bash
# Round 5 29th GPU call: bucket sizes and piece starts in one kernel (k_bucket_finish: one bucket per
# thread, the end offsets from the next lane), one listed-keys atomic per tier workgroup.  The whole GPU suite, configs[1] / configs[2] lines, the
# configs[1] and configs[2] tails (kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05zc; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -ne 0 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, round(d.get("pcie_h2d_GBps") or 0, 2))
PYEOF
}
for rep in 1 2; do
  run c2 X=1 python -u bench.py $B || exit 1
  run c3 X=1 python -u bench.py --workload c3 $B || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_c3/run_kernel_trace.csv > $O/c3_tail.txt && grep -E "bucket_finish|bucket_write|tiers|flags" $O/c3_tail.txt; python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 40 | grep -E "finish|tiers|bucket_write" && tail -1 $O/c3_tail.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c2.json 2> $O/prof_c2.err || { echo "prof failed"; tail -20 $O/prof_c2.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_c2/run_kernel_trace.csv 3 > $O/c2_tail.txt && tail -1 $O/c2_tail.txt
