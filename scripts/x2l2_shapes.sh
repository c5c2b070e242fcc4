#!/bin/bash
# FASTKMER_X2_L2 A/B (0 = by keys per super-cell, 512 = the whole-job kernel everywhere) at the
# configs[3] shape (k = 55) and the configs[2] shape, 1 GB per GPU, host input (gpurun_out/ab.log)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--workload c4 --bytes-per-gpu 1000000000" bash scripts/ab_env.sh FASTKMER_X2_L2 "0 512" || exit 1
BENCH_ARGS="--workload c3 --bytes-per-gpu 1000000000" bash scripts/ab_env.sh FASTKMER_X2_L2 "0 512" || exit 1
