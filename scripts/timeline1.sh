#!/bin/bash
# Kernel + copy timeline of the host-input bench at the default pieces (scripts/timeline.py reads it)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_s -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/tl_s.log 2>&1 || exit 1
