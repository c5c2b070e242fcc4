#!/bin/bash
# Dense compaction with 64 buckets per wave: the full GPU suite, the host-input bench A/B of
# FASTKMER_COMPACT (0 = 64 buckets per wave, 1 = one wave per bucket), rocprof kernel stats of the
# default bench (gpurun_out/cp_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/cp_tests.log 2>&1 \
    || { tail -40 $O/cp_tests.log; exit 1; }
tail -2 $O/cp_tests.log
bash scripts/ab_env.sh FASTKMER_COMPACT "0 1" || exit 1
cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/cp_prof -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/cp_prof.log 2>&1 || exit 1
