#!/bin/bash
# Round 5 34th GPU call (final tree: exchange steps of at least 64 MB): the whole GPU suite, smoke, the default bench line and its kernel stats, and the
# per-GPU-load lines (configs[2] sorted / useHT / one-rank exchange, configs[3] sorted / useHT).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05zh; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 400 --timeout-method thread \
  -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[[ $rc -gt 1 ]] && { echo "suite rc=$rc"; tail -30 $O/suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
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
run c3 X=1 python -u bench.py --workload c3 $B || exit 1
run c3_ht X=1 python -u bench.py --workload c3 --use-ht $B || exit 1
run c3_rehearse1 X=1 python -u bench.py --rehearse-local 1 --workload c3 $B || exit 1
run c4 X=1 python -u bench.py --workload c4 $B || exit 1
run c4_ht X=1 python -u bench.py --workload c4 --use-ht $B || exit 1
run c2_ht X=1 python -u bench.py --use-ht $B || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 5 \
  --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "prof failed"; tail -20 $O/prof_bench.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_bench/run_kernel_stats.csv 8
python3 $R/scripts/kstats.py $O/prof_bench/run_kernel_stats.csv 40 > $O/bench_kernel_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xch1 -o run -- python3 $R/bench.py --workload c3 \
  --rehearse-local 1 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_xch1.json 2> $O/prof_xch1.err || { echo "prof xch failed"; tail -20 $O/prof_xch1.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_xch1/run_kernel_trace.csv > $O/xch1_c3_tail.txt && tail -1 $O/xch1_c3_tail.txt
cd $R
run c2_x1 X=1 python -u bench.py --rehearse-local 1 $B || exit 1
python3 -c "import bench, os; n = bench.pin_to_gpu_numa(0); print('numa node of GPU 0:', n, 'cpus now', len(os.sched_getaffinity(0)))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x1c2 -o run -- python3 $R/bench.py \
  --rehearse-local 1 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_x1c2.json 2> $O/prof_x1c2.err || { echo "prof failed"; tail -20 $O/prof_x1c2.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_x1c2/run_kernel_trace.csv > $O/x1_c2_tail.txt && tail -1 $O/x1_c2_tail.txt
