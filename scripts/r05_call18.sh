#!/bin/bash
# Round 5 18th GPU call: the full-size exchange parity test (1 GB through one and two in-process ranks
# at the product's piece sizes), then the configs[1] tail after the last byte (kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05r; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest "tests/test_gpu_comm.py::test_full_size_exchange_vs_one_count" \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR|assert" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c2.json 2> $O/prof_c2.err || { echo "prof failed"; tail -20 $O/prof_c2.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_c2/run_kernel_trace.csv > $O/c2_tail.txt && tail -45 $O/c2_tail.txt
