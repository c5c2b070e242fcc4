#!/bin/bash
# Kernel profile of the configs[3] rank-0 count at a given job size (GB)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof_c4
FASTKMER_C4_GB=${1:-25} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python -u -m pytest tests/test_gpu_configs.py -k c4_per_gpu -s -q > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
grep "configs\[3\]" gpurun_out/prof_c4.log
python scripts/kstats.py gpurun_out/prof_c4/run_kernel_stats.csv 14
