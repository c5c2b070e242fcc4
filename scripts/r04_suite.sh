#!/bin/bash
# Full GPU suite (every step time-limited; the chain stops at the first failure), then smoke().
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v ${SUITE_ARGS:-} --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -2
