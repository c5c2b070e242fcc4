#!/bin/bash
# Round 6, 37th GPU call: the 64-bit split's first cut stores each key straight into its sub-bucket's 512-key
# region of the split copy (no second pass unless a sub-bucket overflows it): parity suites (+ the
# configs[2]-load tests), A/B lines against lib_prev (the previous commit), and the heavy tiers' per-key
# cost against the wave tier's with every kernel alone (lib_noside, the whole configs[2] load from HBM).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zm; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_wave.py tests/test_gpu_c3_load.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[[ $rc -ne 0 ]] && { echo "gpu tests rc=$rc"; tail -30 $O/gpu_tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
OLD=FASTKMER_LIB=$R/fastkmer_amd/lib_prev/libfastkmer.so
for r in 1 2 3; do
  line c3_new_$r c3 X=1 || exit 1
  line c3_old_$r c3 $OLD || exit 1
done
for r in 1 2; do
  line c2_new_$r c2 X=1 || exit 1
  line c2_old_$r c2 $OLD || exit 1
done
export TMPDIR=/tmp
NS=$R/fastkmer_amd/lib_noside/libfastkmer.so
(cd /tmp && timeout -k 10 300 env FASTKMER_LIB=$NS FK_B=8192 FK_BYTES=6250000000 FK_GENOME=3000000000 FK_JOBS=2 \
  rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
  python3 $R/scripts/count_once.py > $O/prof_c3.log 2>&1) || { echo "prof c3 failed"; tail -5 $O/prof_c3.log; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 30 > $O/kstats_c3.txt
grep -E "^count" $O/prof_c3.log; grep -E "wave<|parts|split|sub_count|mid512|count64<" $O/kstats_c3.txt
