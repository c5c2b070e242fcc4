#!/bin/bash
# Kernel-time profile of one bench workload: bash scripts/prof_bench.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/pb_$tag" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$ROOT/gpurun_out/pb_$tag.log" 2>&1 || exit 1
python3 "$ROOT/scripts/kstats.py" "$ROOT/gpurun_out/pb_$tag/run_kernel_stats.csv" 12
