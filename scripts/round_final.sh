#!/bin/bash
# Full GPU suite, the default bench line, and a rocprofv3 kernel-trace summary of the same bench
# command (gpurun_out/f_*); each step time-limited, the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/f_tests.log 2>&1 || { tail -30 $O/f_tests.log; exit 1; }
tail -2 $O/f_tests.log
timeout -k 10 400 python -u bench.py > $O/f_bench.json 2> $O/f_bench.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/f_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/f_prof.log 2>&1 || exit 1
