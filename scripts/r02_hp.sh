#!/bin/bash
# histogram pieces: GPU suite, configs[2] rehearsal, rank-0 count at N = 1 / 4 / 8 with a kernel profile at 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="-" bash scripts/r02_sort.sh hp || exit 1
FASTKMER_C3_GB=10 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 280 --timeout-method thread \
    -p no:cacheprovider -k per_gpu_load > gpurun_out/c3load10_hp.log 2>&1 || exit 1
grep "configs\[2\]" gpurun_out/c3load10_hp.log
bash scripts/prof_scale.sh hp 8 && python3 scripts/kstats.py gpurun_out/prof_hp/run_kernel_stats.csv 12
