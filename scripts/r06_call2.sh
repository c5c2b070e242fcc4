#!/bin/bash
# Round 6, 2nd GPU call: the RCCL timeout / no-split tests, the k > 32 heavy-bucket split parity tests (and the
# wave / hash / pieces suites), the configs[3] per-GPU load line (k = 55) and its kernel stats, then PMC
# (HBM bytes, VALU, LDS) per kernel at configs[1] and at the configs[2] load.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06b; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -k "rccl" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/comm.log 2>&1
rc=$?; tail -3 $O/comm.log; grep -E "FAILED|ERROR|^E " $O/comm.log | head -20
[[ $rc -gt 1 ]] && { echo "comm rc=$rc"; tail -30 $O/comm.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_hash.py \
  tests/test_gpu_pieces.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -gt 1 ]] && { echo "parity rc=$rc"; tail -30 $O/parity.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
for wl in c4 c3; do
  timeout -k 10 300 python -u bench.py --workload $wl $B > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -5 $O/$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()}, d['buckets_rank0'])" $O/$wl.json $wl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --workload c4 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off > $O/prof_c4.json 2> $O/prof_c4.err || { echo "prof c4 failed"; tail -20 $O/prof_c4.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c4/run_kernel_stats.csv 30 > $O/c4_kernel_stats.txt; head -14 $O/c4_kernel_stats.txt
python3 $R/scripts/tail_timeline.py $O/prof_c4/run_kernel_trace.csv > $O/c4_tail.txt && tail -16 $O/c4_tail.txt
cd $R
timeout -k 10 900 bash scripts/r06_pmc.sh r06b > $O/pmc.log 2>&1; rc=$?; cat $O/pmc.log | grep -v "^c[23] pass"; exit $rc
