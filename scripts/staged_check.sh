#!/bin/bash
# Staged pieces: the pieces tests (both modes), the parity suite's piece-sensitive files, the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/st_tests.log 2>&1 || { tail -40 $O/st_tests.log; exit 1; }
tail -3 $O/st_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/st_bench.json 2> $O/st_bench.err || { tail -20 $O/st_bench.err; exit 1; }
cat $O/st_bench.json
