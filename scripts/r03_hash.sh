#!/bin/bash
# Round 3: useHT LDS tables (large spills, 128-bit keys), the parity suite, the HT benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_parity.py tests/test_distributed.py -k "not rccl" -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_hash_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r03_hash_tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --use-ht > gpurun_out/r03_bench_ht.json 2> gpurun_out/r03_bench_ht.err || { tail -30 gpurun_out/r03_bench_ht.err; exit 1; }
cat gpurun_out/r03_bench_ht.json
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --use-ht --workload c4 --bytes-per-gpu 1000000000 > gpurun_out/r03_bench_ht_c4.json 2> gpurun_out/r03_bench_ht_c4.err || { tail -30 gpurun_out/r03_bench_ht_c4.err; exit 1; }
cat gpurun_out/r03_bench_ht_c4.json
