#!/bin/bash
# Round 5 33rd GPU call: the 513..1024-key buckets through the split + in-order sub-bucket count
# (lib_midsplit, -DFK_MID_SPLIT=1) instead of the mid wave tier: split-parity tests on the variant,
# configs[1] / the configs[2] load (sorted, useHT), alternating; kernel stats of the variant.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05zg; mkdir -p $O
cd $R
FASTKMER_LIB=$R/fastkmer_amd/lib_midsplit/libfastkmer.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_hash.py tests/test_gpu_pieces.py -m gpu -k "not test_block_and_big_tiers" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -ne 0 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, round(d.get("pcie_h2d_GBps") or 0, 2))
PYEOF
}
for v in default midsplit default midsplit; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_$v $L python -u bench.py $B || exit 1
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
  run c3ht_$v $L python -u bench.py --workload c3 --use-ht $B || exit 1
done
cd /tmp && export TMPDIR=/tmp
export FASTKMER_LIB=$R/fastkmer_amd/lib_midsplit/libfastkmer.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 20 | grep -E "count64|split|seq"
