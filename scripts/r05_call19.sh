#!/bin/bash
# Round 5 19th GPU call: the full-size exchange parity test (steps asserted from the 128 MB piece
# floor), then the H2D copy-rate microbenchmark (SDMA and blit-kernel copies, streams, zero-copy).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05s; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest "tests/test_gpu_comm.py::test_full_size_exchange_vs_one_count" \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR|Error" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 ./scripts/ubench/h2d > $O/h2d_sdma.txt 2>&1 && cat $O/h2d_sdma.txt || { echo "h2d failed"; cat $O/h2d_sdma.txt; exit 1; }
export HSA_ENABLE_SDMA=0
timeout -k 10 120 ./scripts/ubench/h2d > $O/h2d_blit.txt 2>&1 && cat $O/h2d_blit.txt || { echo "h2d blit failed"; cat $O/h2d_blit.txt; exit 1; }
