#!/bin/bash
# Round 3: configs[2]/[3] per-GPU loads and configs[4] over 8 ranks; piece profile.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 600 --timeout-method thread \
    > gpurun_out/r03_configs_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|configs\[" gpurun_out/r03_configs_tests.log | tail -15
exit $rc
