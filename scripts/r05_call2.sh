#!/bin/bash
# Round 5 second GPU call: the hash / pieces / comm / split tests after the useHT bucket path and the
# counts communicator; heavy-bucket split A/B at configs[2] (ab/nosplit = the tree before the split);
# useHT on the bucket path vs the group tables at the configs[1..3] loads; configs[2] kernel stats;
# the one-rank exchange rehearsal of configs[2].
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05b; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_pieces.py tests/test_gpu_comm.py \
  tests/test_gpu_write.py tests/test_gpu_wave.py "tests/test_gpu_parity.py::test_heavy_bucket_split_vs_oracle" \
  -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
B="--steps 5 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, d.get("buckets_rank0"))
EOF
}
AB="import sys, runpy; sys.path.insert(0, 'ab/nosplit'); import fastkmer_amd; sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')"
run c3_sorted X=1 python -u bench.py --workload c3 $B || exit 1
run c3_sorted_nosplit X=1 python -u -c "$AB" --workload c3 $B || exit 1
run c3_sorted_b X=1 python -u bench.py --workload c3 $B || exit 1
run c3_ht_buckets X=1 python -u bench.py --workload c3 --use-ht $B || exit 1
run c3_ht_groups FASTKMER_HT_GROUPS=1 python -u bench.py --workload c3 --use-ht $B || exit 1
run c4_sorted X=1 python -u bench.py --workload c4 $B || exit 1
run c4_ht_buckets FASTKMER_BENCH_MEMINFO=1 python -u bench.py --workload c4 --use-ht $B || exit 1
grep meminfo $O/c4_ht_buckets.err
run c4_ht_groups FASTKMER_HT_GROUPS=1 python -u bench.py --workload c4 --use-ht $B || exit 1
run c2_ht_buckets X=1 python -u bench.py --use-ht $B || exit 1
run c2_ht_groups FASTKMER_HT_GROUPS=1 python -u bench.py --use-ht $B || exit 1
run c3_rehearse1 FASTKMER_BENCH_MEMINFO=1 python -u bench.py --rehearse-local 1 --workload c3 $B || exit 1
grep meminfo $O/c3_rehearse1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
find $O/prof_c3 -name "*kernel_stats.csv" | head -3
