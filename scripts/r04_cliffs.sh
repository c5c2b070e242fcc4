#!/bin/bash
# Round-4 first look at the per-GPU loads of configs[2] / configs[3]: rocprofv3 kernel stats of
# bench --workload c3 (6.25 GB), the configs[3] rank-0 test (50 GB job) and bench --workload c4.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_comm.py -k "failing_rank or without_comm or file_range or size_aware" > $O/newtests.log 2>&1 || { tail -30 $O/newtests.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3b -o run -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3b.log 2>&1 || { tail -20 $O/c3b.log; exit 1; }
python3 $R/scripts/kstats.py $O/c3b/run_kernel_stats.csv 25 > $O/c3b_stats.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4t -o run -- python3 -m pytest -x -s -q -p no:cacheprovider $R/tests/test_gpu_configs.py::test_c4_per_gpu_load_rank0_properties > $O/c4t.log 2>&1 || { tail -20 $O/c4t.log; exit 1; }
python3 $R/scripts/kstats.py $O/c4t/run_kernel_stats.csv 25 > $O/c4t_stats.txt
FASTKMER_BENCH_MEMINFO=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4b -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4b.log 2>&1 || { tail -20 $O/c4b.log; exit 1; }
python3 $R/scripts/kstats.py $O/c4b/run_kernel_stats.csv 25 > $O/c4b_stats.txt
