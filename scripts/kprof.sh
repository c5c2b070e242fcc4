#!/bin/bash
# Kernel-time profile of scripts/count_once.py under the given env assignments:
#   bash scripts/kprof.sh TAG [VAR=val ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); tag=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/kp_$tag" -o run --output-format csv \
    -- python3 "$ROOT/scripts/count_once.py" > "$ROOT/gpurun_out/kp_$tag.log" 2>&1 || exit 1
python3 "$ROOT/scripts/kstats.py" "$ROOT/gpurun_out/kp_$tag/run_kernel_stats.csv" 14
