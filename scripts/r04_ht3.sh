#!/bin/bash
# useHT=1, third pass: 512-thread 128-bit combine (default), heavy-group tables (FASTKMER_HT_BIG) with
# 1024- and 512-thread workgroups (lib_htbig512), the 64-bit combine at 512 threads (lib_ht64n512)
# at configs[1]; c4-shape bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/ht3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hash.py tests/test_gpu_write.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
probe() {  # name lib env...
  local n=$1 l=$2; shift 2
  if [ $l = base ]; then unset FASTKMER_LIB; else export FASTKMER_LIB=$R/fastkmer_amd/lib_$l/libfastkmer.so; fi
  env "$@" timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_$n.txt 2>&1 || { tail -20 $O/probe_$n.txt; exit 1; }
  echo "== $n"; grep LDS $O/probe_$n.txt
}
probe base base FK_X=0 || exit 1
probe big1800 base FASTKMER_HT_BIG=1800 || exit 1
probe big1300 base FASTKMER_HT_BIG=1300 || exit 1
probe big512_1800 htbig512 FASTKMER_HT_BIG=1800 || exit 1
probe big512_1300 htbig512 FASTKMER_HT_BIG=1300 || exit 1
unset FASTKMER_LIB
for v in base ht64n512; do
  if [ $v = base ]; then unset FASTKMER_LIB; else export FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so; fi
  timeout -k 10 300 python -u bench.py --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c1_ht_$v.json 2> $O/bench_c1_ht_$v.err || { tail -20 $O/bench_c1_ht_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stages_ms'], d.get('device_resident_stages_ms'))" $O/bench_c1_ht_$v.json c1_ht_$v
done
unset FASTKMER_LIB
FASTKMER_HT_BIG=1800 timeout -k 10 300 python -u bench.py --workload c4 --bytes-per-gpu 1000000000 --use-ht --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4_1g_ht.json 2> $O/bench_c4_1g_ht.err || { tail -20 $O/bench_c4_1g_ht.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4_1g_ht_big1800', d['ms_per_step'], d['stages_ms'], d.get('device_resident_stages_ms'))" $O/bench_c4_1g_ht.json
