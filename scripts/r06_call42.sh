#!/bin/bash
# Round 6, 42nd GPU call (round-end tree: + the key-range mid tier's keys in registers, the 128-bit four-piece test): the whole GPU suite, smoke, the default bench line, its kernel stats
# under rocprofv3 (the graded map kernel's launches), the configs[3] per-GPU load line, the one-rank exchange
# lines at the configs[2] / configs[3] loads and useHT at the configs[3] load.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zr; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[[ $rc -gt 1 ]] && { echo "suite rc=$rc"; tail -30 $O/suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(d['value']/1e9,2), 'Gbases/s', round(d['ms_per_step'],2), 'ms; roofline', round(d['roofline']['frac'],4), d['roofline']['ms_per_launch']); print('c3 leg', round(d['configs2_per_gpu']['ms_per_step'],2))" $O/bench.json
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py \
  --steps 5 --warmup 2 --no-cpu-baseline --c3-leg off > $O/prof_bench.json 2> $O/prof_bench.err) || { echo "prof bench failed"; tail -20 $O/prof_bench.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_bench/run_kernel_stats.csv 30 > $O/bench_kernel_stats.txt; head -6 $O/bench_kernel_stats.txt
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name, then bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
line c4 --workload c4 || exit 1
line c4_rehearse1 --workload c4 --rehearse-local 1 || exit 1
line c3_rehearse1 --workload c3 --rehearse-local 1 || exit 1
line c4_ht --workload c4 --use-ht || exit 1
line c3_ht --workload c3 --use-ht || exit 1
line c3 --workload c3 || exit 1
python3 - $O/prof_bench/run_kernel_trace.csv > $O/map_launches.txt <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_map_fused" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
whole = [x for x in d if x > 0.9]
print(f"k_map_fused launches {len(d)}; whole-input (> 0.9 ms) {len(whole)}: mean {statistics.mean(whole) if whole else 0:.4f} ms "
      f"min {min(whole) if whole else 0:.4f} max {max(whole) if whole else 0:.4f}")
PY
cat $O/map_launches.txt
