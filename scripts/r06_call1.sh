#!/bin/bash
# Round 6, 1st GPU call: the comm tests (bounded waits, FASTKMER_COMM_SPLIT=0), the configs[2] per-GPU load
# on the bench's own path vs the bin-filtered oracle and the one-rank exchange vs the whole-input count,
# smoke, and the kernel stats / tail timeline of the configs[3] per-GPU load (k = 55).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06a; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/comm.log 2>&1
rc=$?; tail -3 $O/comm.log; grep -E "FAILED|ERROR" $O/comm.log | head -20
[[ $rc -gt 1 ]] && { echo "comm rc=$rc"; tail -30 $O/comm.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/wave_parity.log 2>&1
rc=$?; tail -3 $O/wave_parity.log; grep -E "FAILED|ERROR" $O/wave_parity.log | head -20
[[ $rc -gt 1 ]] && { echo "wave/parity rc=$rc"; tail -30 $O/wave_parity.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_c3_load.py -v -s --timeout 900 --timeout-method thread \
  -p no:cacheprovider > $O/c3_load.log 2>&1
rc=$?; grep -E "c3-load|passed|failed|FAILED|Error" $O/c3_load.log | tail -20
[[ $rc -gt 1 ]] && { echo "c3 load rc=$rc"; tail -30 $O/c3_load.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --workload c4 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c4.json 2> $O/prof_c4.err || { echo "prof c4 failed"; tail -20 $O/prof_c4.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c4/run_kernel_stats.csv 30 > $O/c4_kernel_stats.txt; head -16 $O/c4_kernel_stats.txt
python3 $R/scripts/tail_timeline.py $O/prof_c4/run_kernel_trace.csv > $O/c4_tail.txt && tail -25 $O/c4_tail.txt
