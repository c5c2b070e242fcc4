#!/bin/bash
# useHT=1 round 2 of measurements: spill rounds planned on the device; round-1 probes (lib_htp1: no
# inserts, lib_htp2: no inserts and no output, both wrong results by design) and a 512-thread
# combine (lib_htn512); kernel trace of the product run; c4-shape bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/ht2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hash.py tests/test_gpu_write.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in base htn512 htp1 htp2; do
  if [ $v = base ]; then unset FASTKMER_LIB; else export FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so; fi
  timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_$v.txt 2>&1 || { tail -20 $O/probe_$v.txt; exit 1; }
  echo "== $v"; cat $O/probe_$v.txt | grep LDS
done
unset FASTKMER_LIB
for t in 1800 2600; do
  FASTKMER_HT_BIG=$t timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_big$t.txt 2>&1 || { tail -20 $O/probe_big$t.txt; exit 1; }
  echo "== big $t"; grep LDS $O/probe_big$t.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/scripts/ht_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 $R/scripts/kstats.py $O/p/run_kernel_stats.csv 20
cd $R
timeout -k 10 300 python -u bench.py --workload c4 --bytes-per-gpu 1000000000 --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4_1g_ht.json 2> $O/bench_c4_1g_ht.err || { tail -20 $O/bench_c4_1g_ht.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'], d.get('device_resident_stages_ms'))" $O/bench_c4_1g_ht.json
