#!/bin/bash
# Round 3: native exchange (fk_comm_*) GPU tests, then the bench legs (N = 1 and local rehearsals).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_comm_tests.log 2>&1 || { tail -50 gpurun_out/r03_comm_tests.log; exit 1; }
tail -5 gpurun_out/r03_comm_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_n1.json 2> gpurun_out/r03_bench_n1.err || { tail -30 gpurun_out/r03_bench_n1.err; exit 1; }
cat gpurun_out/r03_bench_n1.json
timeout -k 10 300 python -u bench.py --rehearse-local 2 --bytes-per-gpu 1000000000 --steps 3 --warmup 1 > gpurun_out/r03_rehearse2.json 2> gpurun_out/r03_rehearse2.err || { tail -30 gpurun_out/r03_rehearse2.err; exit 1; }
cat gpurun_out/r03_rehearse2.json
timeout -k 10 300 python -u bench.py --rehearse-local 8 --bytes-per-gpu 400000000 --steps 3 --warmup 1 > gpurun_out/r03_rehearse8.json 2> gpurun_out/r03_rehearse8.err || { tail -30 gpurun_out/r03_rehearse8.err; exit 1; }
cat gpurun_out/r03_rehearse8.json
