#!/bin/bash
# (second run, r06zh: r06zg failed the configs[2]-load test on its large-path assertion -- the second cut left no bucket to it)
# Round 6, 32nd GPU call: split buckets whose cut left a sub-bucket above 512 keys cut again (twice the
# sub-buckets, another sample) with the heavy tiers' stream at the highest priority, against lib_prio0 (neither):
# parity / pieces / wave suites (the retry hook's split tests), A/B lines, the configs[2]-load and configs[1] tails.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zh; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_wave.py tests/test_gpu_c3_load.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[[ $rc -ne 0 ]] && { echo "gpu tests rc=$rc"; tail -30 $O/gpu_tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P0=FASTKMER_LIB=$R/fastkmer_amd/lib_prio0/libfastkmer.so
for r in 1 2 3; do
  line c2_hi_$r c2 X=1 || exit 1
  line c2_p0_$r c2 $P0 || exit 1
  line c3_hi_$r c3 X=1 || exit 1
  line c3_p0_$r c3 $P0 || exit 1
done
for r in 1 2; do
  line c4_hi_$r c4 X=1 || exit 1
  line c4_p0_$r c4 $P0 || exit 1
done
export TMPDIR=/tmp
for wl in c3 c2; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 $R/bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$wl.json 2> $O/prof_$wl.err) || { echo "prof $wl failed"; tail -5 $O/prof_$wl.err; exit 1; }
  python3 $R/scripts/tail_timeline.py $O/prof_$wl/run_kernel_trace.csv > $O/tail_$wl.txt
  echo "== $wl"; tail -1 $O/tail_$wl.txt
done
