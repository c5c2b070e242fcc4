#!/bin/bash
# 128-bit (k = 55) count: parity tests, then configs[3]'s per-GPU load (rank-0 test, bench line)
# with the mid wave tier (default) and without it (FASTKMER_MID128=0), kernel stats of each.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "55 or 128 or k55 or two_word or c4 or wave" > $O/c4_tests.log 2>&1 || { tail -30 $O/c4_tests.log; exit 1; }
tail -2 $O/c4_tests.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  FASTKMER_MID128=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4t$v -o run -- python3 -m pytest -x -s -q -p no:cacheprovider $R/tests/test_gpu_configs.py::test_c4_per_gpu_load_rank0_properties > $O/c4t$v.log 2>&1 || { tail -20 $O/c4t$v.log; exit 1; }
  python3 $R/scripts/kstats.py $O/c4t$v/run_kernel_stats.csv 16 > $O/c4t${v}_stats.txt
  FASTKMER_MID128=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4b$v -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4b$v.log 2>&1 || { tail -20 $O/c4b$v.log; exit 1; }
  python3 $R/scripts/kstats.py $O/c4b$v/run_kernel_stats.csv 16 > $O/c4b${v}_stats.txt
done
