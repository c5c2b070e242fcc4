#!/bin/bash
# Round 5 tenth GPU call: the whole GPU suite, smoke, the default bench line, its kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05j; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 400 --timeout-method thread \
  -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[[ $rc -gt 1 ]] && { echo "suite rc=$rc"; tail -30 $O/suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 5 \
  --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "prof failed"; tail -20 $O/prof_bench.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_bench/run_kernel_stats.csv 12
grep -o '"roofline": {[^}]*}' $O/prof_bench.json
