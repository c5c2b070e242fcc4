#!/bin/bash
# Round 6, 21st GPU call: the 64-bit mid tier as 2-3 key ranges on the wave tier's table (k_bucket_count64_parts,
# FK_MID_PARTS default; lib_noparts = every mid bucket on the 1024-key kernel): parity (the new ranges test with
# repeated reads, the heavy / block / pieces / wave suites), A/B lines, kernel stats at the configs[2] load.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06v; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k mid_tier \
  -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -ne 0 ]] && { echo "parity rc=$rc"; grep -E "^E " $O/parity.log | head -30; exit 1; }
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
NP=FASTKMER_LIB=$R/fastkmer_amd/lib_noparts/libfastkmer.so
for r in 1 2; do
  line c3_parts$r c3 X=1 || exit 1
  line c3_noparts$r c3 $NP || exit 1
  line c2_parts$r c2 X=1 || exit 1
  line c2_noparts$r c2 $NP || exit 1
done
export TMPDIR=/tmp
for v in parts noparts; do
  E=X=1; [[ $v == noparts ]] && E=$NP
  (cd /tmp && timeout -k 10 240 env $E rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
    python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$v.json 2> $O/prof_$v.err) || { echo "prof $v failed"; tail -5 $O/prof_$v.err; exit 1; }
  python3 $R/scripts/kstats.py $O/prof_$v/run_kernel_stats.csv 40 > $O/kstats_$v.txt
  python3 $R/scripts/tail_timeline.py $O/prof_$v/run_kernel_trace.csv > $O/tail_$v.txt
  echo "== $v: $(tail -1 $O/tail_$v.txt)"; grep -E "count64_wave|count64_parts|split64|sub_count64" $O/kstats_$v.txt
done
