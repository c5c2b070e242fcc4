#!/bin/bash
# Round 6, 10th GPU call: rank member loops read 4 (64-bit) / 2 (128-bit) members per LDS round trip, the
# in-order sub-bucket count's prefetch not branched over, the split's key loads from one base per row;
# parity of the product library, A/B lines against lib_base6, kernel stats and the tail after the last
# byte at the configs[2] and configs[3] loads.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06j; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_pieces.py \
  tests/test_gpu_hash.py tests/test_gpu_c3_load.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -gt 1 ]] && { echo "parity rc=$rc"; tail -30 $O/parity.log; exit 1; }
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
OLD=FASTKMER_LIB=$R/fastkmer_amd/lib_base6/libfastkmer.so
for r in 1 2; do
  line c3_old$r c3 $OLD || exit 1
  line c3_new$r c3 X=1 || exit 1
  line c4_old$r c4 $OLD || exit 1
  line c4_new$r c4 X=1 || exit 1
  line c2_old$r c2 $OLD || exit 1
  line c2_new$r c2 X=1 || exit 1
done
export TMPDIR=/tmp
for wl in c3 c4; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 $R/bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$wl.json 2> $O/prof_$wl.err) || { echo "prof $wl failed"; tail -5 $O/prof_$wl.err; exit 1; }
  python3 $R/scripts/kstats.py $O/prof_$wl/run_kernel_stats.csv 40 > $O/kstats_$wl.txt
  python3 $R/scripts/tail_timeline.py $O/prof_$wl/run_kernel_trace.csv > $O/tail_$wl.txt
  echo "== $wl"; head -12 $O/kstats_$wl.txt; tail -1 $O/tail_$wl.txt
done
