#!/bin/bash
# Round 5 24th GPU call: split buckets' sub-buckets counted in order by one wave per bucket straight
# into the bucket's output (no join) vs the sub-bucket wave + join (lib_subjoin).  Parity tests of
# the split / hash / pieces / write paths, then the configs[2] load (sorted, useHT) and configs[1] A/B,
# kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05x; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hash.py tests/test_gpu_pieces.py tests/test_gpu_write.py \
  tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
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
for v in default subjoin default subjoin; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
  run c3ht_$v $L python -u bench.py --workload c3 --use-ht $B || exit 1
  run c2_$v $L python -u bench.py $B || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 16 | grep -E "count64|split|join|seq"
