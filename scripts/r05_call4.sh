#!/bin/bash
# Round 5 fourth GPU call: the heavy-split parity cases; configs[2] / [1] with and without the heavy
# split (lib_nosplit = -DFK_SPLIT_HEAVY=0); useHT; the one-rank exchange with staging on its own
# stream; the two-rank configs[2] rehearsal on one GPU (footprint); kernel stats; PMC of the tiers.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05d; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_heavy_bucket_split_vs_oracle" tests/test_gpu_comm.py \
  -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 5 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, d.get("buckets_rank0"))
PYEOF
}
NS=FASTKMER_LIB=$R/fastkmer_amd/lib_nosplit/libfastkmer.so
run c3_sorted X=1 python -u bench.py --workload c3 $B || exit 1
run c3_sorted_nosplit $NS python -u bench.py --workload c3 $B || exit 1
run c2_sorted X=1 python -u bench.py $B || exit 1
run c2_sorted_nosplit $NS python -u bench.py $B || exit 1
run c3_ht X=1 python -u bench.py --workload c3 --use-ht $B || exit 1
run c3_rehearse1 FASTKMER_BENCH_MEMINFO=1 python -u bench.py --rehearse-local 1 --workload c3 $B || exit 1
grep meminfo $O/c3_rehearse1.err
run c3_rehearse2 FASTKMER_BENCH_MEMINFO=1 python -u bench.py --rehearse-local 2 --workload c3 --bytes-per-gpu 6250000000 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg || echo "rehearse2 failed (see above)"
grep meminfo $O/c3_rehearse2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xch1 -o run -- python3 $R/bench.py --workload c3 \
  --rehearse-local 1 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_xch1.json 2> $O/prof_xch1.err || { echo "prof xch failed"; tail -20 $O/prof_xch1.err; exit 1; }
cd $R
bash scripts/r05_pmc_wave.sh r05d || exit 1
