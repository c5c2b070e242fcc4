#!/bin/bash
# Round-4 measurements: headline bench with / without the pre-count, rocprofv3 kernel stats of the
# headline bench, then the per-GPU loads of configs[2] / configs[3] (bench lines + kernel stats, the
# configs[3] rank-0 test).  Every step time-limited; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/m_bench.json 2> $O/m_bench.err || { tail -20 $O/m_bench.err; exit 1; }
FASTKMER_PRECOUNT=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/m_bench_nopre.json 2> $O/m_bench_nopre.err || { tail -20 $O/m_bench_nopre.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/m_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/m_prof.log 2>&1 || { tail -20 $O/m_prof.log; exit 1; }
python3 $R/scripts/kstats.py $O/m_prof/run_kernel_stats.csv 30 > $O/m_prof_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3b -o run -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3b.log 2>&1 || { tail -20 $O/c3b.log; exit 1; }
python3 $R/scripts/kstats.py $O/c3b/run_kernel_stats.csv 30 > $O/c3b_stats.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4t -o run -- python3 -m pytest -x -s -q -p no:cacheprovider $R/tests/test_gpu_configs.py::test_c4_per_gpu_load_rank0_properties > $O/c4t.log 2>&1 || { tail -20 $O/c4t.log; exit 1; }
python3 $R/scripts/kstats.py $O/c4t/run_kernel_stats.csv 30 > $O/c4t_stats.txt
FASTKMER_BENCH_MEMINFO=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4b -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4b.log 2>&1 || { tail -20 $O/c4b.log; exit 1; }
python3 $R/scripts/kstats.py $O/c4b/run_kernel_stats.csv 30 > $O/c4b_stats.txt
