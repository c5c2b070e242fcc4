#!/bin/bash
# Round 3 (b): full GPU suite, then the map phase probes and the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/c_tests.log 2>&1 || { tail -30 $O/c_tests.log; exit 1; }
tail -3 $O/c_tests.log
bash scripts/r03_map_probe.sh > $O/c_map_probe.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/c_bench.json 2> $O/c_bench.err || exit 1
