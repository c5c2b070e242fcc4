#!/bin/bash
# Round-4 end: full GPU suite + smoke (r04_suite.sh), the default bench line, rocprofv3 kernel stats of
# the same bench, the useHT bench lines (configs[1], configs[3] shape at 1 GB) and the useHT kernel
# stats at the configs[3] shape.  Every step time-limited; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/fin; mkdir -p $O
cd $R
bash scripts/r04_suite.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c1_ht.json 2> $O/bench_c1_ht.err || { tail -20 $O/bench_c1_ht.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --bytes-per-gpu 1000000000 --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4_1g_ht.json 2> $O/bench_c4_1g_ht.err || { tail -20 $O/bench_c4_1g_ht.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --bytes-per-gpu 1000000000 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4_1g_sorted.json 2> $O/bench_c4_1g_sorted.err || { tail -20 $O/bench_c4_1g_sorted.err; exit 1; }
for f in bench_c1_ht bench_c4_1g_ht bench_c4_1g_sorted; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stages_ms'], d.get('device_resident_stages_ms'))" $O/$f.json $f
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 $R/scripts/kstats.py $O/prof/run_kernel_stats.csv 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/htp -o run -- python3 $R/scripts/ht_probe.py > $O/htp.log 2>&1 || { tail -20 $O/htp.log; exit 1; }
grep LDS $O/htp.log
python3 $R/scripts/kstats.py $O/htp/run_kernel_stats.csv 12
