#!/bin/bash
# Round 5 twelfth GPU call: the wave rank's group count and cursor packed in one word (parity), and
# 640-slot wave tables (lib_sl640, 7.4 KB per wave: 6 waves per SIMD instead of 5) vs 768.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05l; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_hash.py \
  -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()})
PYEOF
}
for v in default sl640 default sl640; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_$v $L python -u bench.py $B || exit 1
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
done
