#!/bin/bash
# useHT=1 at the configs[3] shape (k=55 m=12 B=8192, 1 GB of 150 bp reads): the hash-count tests,
# per-round count figures (ht_probe.py) with the product library and the round-3 expansion
# (lib_htold, -DFK_HT_PERKMER=0), and rocprofv3 kernel stats of the product run.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/ht; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hash.py tests/test_gpu_write.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
FASTKMER_LIB=$R/fastkmer_amd/lib_htold/libfastkmer.so timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_old.txt 2>&1 || { tail -20 $O/probe_old.txt; exit 1; }
cat $O/probe_old.txt
FASTKMER_HT_SUBPART=0 timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_nosub.txt 2>&1 || { tail -20 $O/probe_nosub.txt; exit 1; }
cat $O/probe_nosub.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/scripts/ht_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 $R/scripts/kstats.py $O/p/run_kernel_stats.csv 16
cd $R
for v in ht sorted; do
  f=""; [ $v = ht ] && f="--use-ht"
  timeout -k 10 300 python -u bench.py --workload c4 --bytes-per-gpu 1000000000 $f --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4_1g_$v.json 2> $O/bench_c4_1g_$v.err || { tail -20 $O/bench_c4_1g_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stages_ms'], d.get('device_resident_stages_ms'))" $O/bench_c4_1g_$v.json $v
done
