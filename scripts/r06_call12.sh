#!/bin/bash
# Round 6, 12th GPU call: the 64-bit rank's final loop over rows of keys with their reads batched
# (FK_W64_RANKV=2, RB = 2 / 4 rows: lib_rankv2b2 / lib_rankv2b4): parity, the wave tier per launch at the
# configs[2] load against the product library and a stop-before-the-final-loop probe (lib_w64stop3), lines.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06l; mkdir -p $O
cd $R
for v in b2 b4; do
  FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2$v/libfastkmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_wave.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/parity_$v.log)"; grep -E "FAILED|ERROR" $O/parity_$v.log | head -10
  [[ $rc -gt 1 ]] && { echo "parity $v rc=$rc"; tail -30 $O/parity_$v.log; exit 1; }
done
export TMPDIR=/tmp
probe() {  # name, then env assignments
  local name=$1; shift
  (cd /tmp && timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
    python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$name.json 2> $O/prof_$name.err) || { echo "probe $name failed"; tail -5 $O/prof_$name.err; return 1; }
  python3 $R/scripts/kstats.py $O/prof_$name/run_kernel_stats.csv 40 > $O/kstats_$name.txt
  echo "$name: $(grep -E 'count64_wave<2' $O/kstats_$name.txt | head -1)"
}
probe full X=1 || exit 1
probe stop3 FASTKMER_LIB=$R/fastkmer_amd/lib_w64stop3/libfastkmer.so || exit 1
probe b2 FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2b2/libfastkmer.so || exit 1
probe b4 FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2b4/libfastkmer.so || exit 1
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
for r in 1 2; do
  line c3_prod$r c3 X=1 || exit 1
  line c3_b2_$r c3 FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2b2/libfastkmer.so || exit 1
  line c3_b4_$r c3 FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2b4/libfastkmer.so || exit 1
  line c2_prod$r c2 X=1 || exit 1
  line c2_b2_$r c2 FASTKMER_LIB=$R/fastkmer_amd/lib_rankv2b2/libfastkmer.so || exit 1
done
