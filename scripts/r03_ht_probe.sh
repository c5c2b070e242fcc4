#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u scripts/ht_probe.py || exit 1
FASTKMER_LDS_HT=0 timeout -k 10 200 python -u scripts/ht_probe.py || exit 1
timeout -k 10 200 python -u scripts/ht_probe.py 28 10 8192 100 || exit 1
mkdir -p gpurun_out/prof_ht
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ht -o run --output-format csv -- python -u scripts/ht_probe.py > gpurun_out/prof_ht.log 2>&1 || exit 1
python scripts/kstats.py gpurun_out/prof_ht/run_kernel_stats.csv 12
