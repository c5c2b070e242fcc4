#!/bin/bash
# Round 6, 3rd GPU call: RCCL bounded-wait tests (pinned staging), the 128-bit fingerprint wave tier's parity
# (incl. forced fingerprint collisions) and an A/B of the configs[3] per-GPU load line against the
# uniform-round dedupe (FK_W128_FP=0, fastkmer_amd/lib_w128old).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06c; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -k "rccl" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/comm.log 2>&1
rc=$?; tail -3 $O/comm.log; grep -E "FAILED|ERROR|^E " $O/comm.log | head -20
[[ $rc -gt 1 ]] && { echo "comm rc=$rc"; tail -30 $O/comm.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_hash.py \
  tests/test_gpu_pieces.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -gt 1 ]] && { echo "parity rc=$rc"; tail -30 $O/parity.log; exit 1; }
B="--steps 6 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name, then env assignments
  local name=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --workload c4 $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
for r in 1 2; do
  line c4_fp$r X=1 || exit 1
  line c4_old$r FASTKMER_LIB=$R/fastkmer_amd/lib_w128old/libfastkmer.so || exit 1
done
timeout -k 10 300 python -u bench.py --workload c4 --use-ht $B > $O/c4ht.json 2> $O/c4ht.err && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4ht', round(d['ms_per_step'],2), d['stages_ms'])" $O/c4ht.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --workload c4 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off > $O/prof_c4.json 2> $O/prof_c4.err || { echo "prof c4 failed"; tail -20 $O/prof_c4.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c4/run_kernel_stats.csv 30 > $O/c4_kernel_stats.txt; head -8 $O/c4_kernel_stats.txt
python3 $R/scripts/tail_timeline.py $O/prof_c4/run_kernel_trace.csv > $O/c4_tail.txt && tail -12 $O/c4_tail.txt
