#!/bin/bash
# Kernel + copy timeline (scripts/timeline.py reads it) of the host-input bench (pieces at the default cut and none)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_p -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/tl_p.log 2>&1 || exit 1
FASTKMER_PIECE_COUNT=0 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_n -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/tl_n.log 2>&1 || exit 1
