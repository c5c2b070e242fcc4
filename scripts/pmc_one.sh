#!/bin/bash
# One rocprofv3 PMC pass over scripts/count_once.py: bash scripts/pmc_one.sh TAG "COUNTERS..." [VAR=val ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); tag=$1; ctr=$2; shift 2
for kv in "$@"; do export "$kv"; done
mkdir -p "$ROOT/gpurun_out/pmc_$tag/p1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$ROOT/gpurun_out/pmc_$tag/p1" -o run --output-format csv \
    -- python3 "$ROOT/scripts/count_once.py" > "$ROOT/gpurun_out/pmc_$tag/p1.log" 2>&1 || exit 1
python3 "$ROOT/scripts/pmc_kernels.py" "$ROOT/gpurun_out/pmc_$tag" bucket_count64 expand_scatter part_scatter
