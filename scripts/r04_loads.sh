#!/bin/bash
# Per-GPU loads of the 8-GPU configs on one GPU: configs[2] (6.25 GB, k=28 B=8192) N=1 and through the
# exchange path with one in-process rank; configs[3] (6.25 GB, k=55) N=1 under rocprofv3 kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/loads; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cat $O/c3.json
FASTKMER_BENCH_MEMINFO=1 timeout -k 10 400 python -u bench.py --rehearse-local 1 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl1c3.json 2> $O/rl1c3.err || { tail -20 $O/rl1c3.err; exit 1; }
cat $O/rl1c3.json; grep meminfo $O/rl1c3.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4p -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
grep metric $O/c4p.log
python3 $R/scripts/kstats.py $O/c4p/run_kernel_stats.csv 16
