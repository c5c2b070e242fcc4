#!/bin/bash
# Round 6, 16th GPU call: the last staged piece's bucket cut on the side stream beside its expansion (FK_CUT_SIDE,
# default; lib_nocutside = after it): parity of the product library (whole GPU suite), A/B lines against
# lib_nocutside and lib_base6 at configs[1] and the configs[2] / configs[3] loads, the configs[2] tail.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06p; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; tail -2 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[[ $rc -ne 0 ]] && { echo "suite rc=$rc"; tail -30 $O/suite.log; exit 1; }
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
NS=FASTKMER_LIB=$R/fastkmer_amd/lib_nocutside/libfastkmer.so
OLD=FASTKMER_LIB=$R/fastkmer_amd/lib_base6/libfastkmer.so
for r in 1 2; do
  line c3_cut$r c3 X=1 || exit 1
  line c3_nocut$r c3 $NS || exit 1
  line c4_cut$r c4 X=1 || exit 1
  line c4_nocut$r c4 $NS || exit 1
  line c2_cut$r c2 X=1 || exit 1
  line c2_nocut$r c2 $NS || exit 1
done
line c3_old c3 $OLD || exit 1
line c4_old c4 $OLD || exit 1
line c2_old c2 $OLD || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
  python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
  > $O/prof_c3.json 2> $O/prof_c3.err) || { echo "prof c3 failed"; tail -5 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 40 > $O/kstats_c3.txt
python3 $R/scripts/tail_timeline.py $O/prof_c3/run_kernel_trace.csv > $O/tail_c3.txt; tail -1 $O/tail_c3.txt
