#!/bin/bash
# Round 3 (b): map phase probes, bench on HEAD, kernel stats of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash scripts/r03_map_probe.sh > $O/b_map_probe.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b_bench.json 2> $O/b_bench.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/b_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/$O/b_prof.log 2>&1 || exit 1
