#!/bin/bash
# Round 6, 34th GPU call: the wave tiers' staged-piece key rows from per-bucket row bases (lane r works out
# row r's piece base once; a row takes it with two lane reads; no branch on the lane's bounds) against
# lib_prev (the previous commit: ~25 scalar instructions per row): parity / pieces / wave suites, A/B lines.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zj; mkdir -p $O
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
OLD=FASTKMER_LIB=$R/fastkmer_amd/lib_prev/libfastkmer.so
for r in 1 2 3 4; do
  line c2_new_$r c2 X=1 || exit 1
  line c2_old_$r c2 $OLD || exit 1
done
for r in 1 2 3; do
  line c3_new_$r c3 X=1 || exit 1
  line c3_old_$r c3 $OLD || exit 1
done
for r in 1 2; do
  line c4_new_$r c4 X=1 || exit 1
  line c4_old_$r c4 $OLD || exit 1
done
