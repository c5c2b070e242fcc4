#!/bin/bash
# Round 6, 33rd GPU call: the 64-bit mid tier of a job whose k-mers repeat (configs[1]: 59 K mid buckets) whole on
# the wave tier's 512-key table (k_bucket_count64_mid512; more than 512 distinct keys: the 1024-key kernel),
# first on the side stream, against the 1024-key kernel for all (FASTKMER_DEBUG_MID_PARTS=0, the previous
# configs[1] path): parity / pieces / wave suites, A/B lines at configs[1] and the configs[2] load, the tails.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zi; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_wave.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[[ $rc -ne 0 ]] && { echo "gpu tests rc=$rc"; tail -30 $O/gpu_tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
OLD=FASTKMER_DEBUG_MID_PARTS=0
for r in 1 2 3 4; do
  line c2_m512_$r c2 X=1 || exit 1
  line c2_m1024_$r c2 $OLD || exit 1
done
for r in 1 2; do
  line c3_new_$r c3 X=1 || exit 1
done
export TMPDIR=/tmp
for wl in c2; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 $R/bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$wl.json 2> $O/prof_$wl.err) || { echo "prof $wl failed"; tail -5 $O/prof_$wl.err; exit 1; }
  python3 $R/scripts/tail_timeline.py $O/prof_$wl/run_kernel_trace.csv > $O/tail_$wl.txt
  echo "== $wl"; tail -1 $O/tail_$wl.txt
done
