#!/bin/bash
# Round 3: per-piece counts + merge (one rank and ranks), the existing GPU suite, the N = 1 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_comm.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pieces_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r03_pieces_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_n1.json 2> gpurun_out/r03_bench_n1.err || { tail -30 gpurun_out/r03_bench_n1.err; exit 1; }
cat gpurun_out/r03_bench_n1.json
