#!/bin/bash
# Round 5 fifth GPU call: parity of the heavy-split / large-path / repeat cases and the exchange after the
# compact large-bucket scratch and the split's cached sub-buckets; configs[2] load, configs[1] headline
# and the two-rank configs[2] rehearsal (footprint); kernel stats of configs[2].
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05e; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_hash.py \
  -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 5 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, d.get("buckets_rank0"))
PYEOF
}
run c3_sorted X=1 python -u bench.py --workload c3 $B || exit 1
run c2_sorted X=1 python -u bench.py $B || exit 1
run c2_nosplit FASTKMER_LIB=$R/fastkmer_amd/lib_nosplit/libfastkmer.so python -u bench.py $B || exit 1
run c3_rehearse1 FASTKMER_BENCH_MEMINFO=1 python -u bench.py --rehearse-local 1 --workload c3 $B || exit 1
grep meminfo $O/c3_rehearse1.err
run c3_rehearse2 FASTKMER_BENCH_MEMINFO=1 python -u bench.py --rehearse-local 2 --workload c3 --bytes-per-gpu 6250000000 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg || echo "rehearse2 failed (see above)"
grep meminfo $O/c3_rehearse2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 16
