#!/bin/bash
# Round 6, 41st GPU call: the split's target keys per sub-bucket (FK_SPL_TGT 256 / 288 / 320; larger sub-buckets,
# fewer per-sub-bucket rounds in the in-order count, more second cuts): configs[2]-load lines and every kernel
# alone at that load (lib_noside / lib_nst288 / lib_nst320), plus the heavy-split parity tests on the 320 build.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zq; mkdir -p $O
cd $R
FASTKMER_LIB=$R/fastkmer_amd/lib_t320/libfastkmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "heavy or mid_tier" \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[[ $rc -ne 0 ]] && { echo "gpu tests rc=$rc"; tail -30 $O/gpu_tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
for r in 1 2; do
  line c3_256_$r c3 X=1 || exit 1
  line c3_288_$r c3 FASTKMER_LIB=$R/fastkmer_amd/lib_t288/libfastkmer.so || exit 1
  line c3_320_$r c3 FASTKMER_LIB=$R/fastkmer_amd/lib_t320/libfastkmer.so || exit 1
done
export TMPDIR=/tmp
for v in noside nst288 nst320; do
  (cd /tmp && timeout -k 10 300 env FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so FK_B=8192 FK_BYTES=6250000000 \
    FK_GENOME=3000000000 FK_JOBS=2 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
    python3 $R/scripts/count_once.py > $O/prof_$v.log 2>&1) || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 $R/scripts/kstats.py $O/prof_$v/run_kernel_stats.csv 30 > $O/kstats_$v.txt
  echo "== $v"; grep -E "^count" $O/prof_$v.log | cut -c1-60; grep -E "wave<|parts|split|sub_count|count64<" $O/kstats_$v.txt
done
