#!/bin/bash
# Round 6, 20th GPU call: the largest-F parity test (cell target set by the test), then PMC per kernel (HBM bytes,
# VALU, LDS) at configs[1] and at the configs[2] load on the round-end tree (scripts/r06_pmc.sh r06t).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06t; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "max_fine_bits" -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/maxf.log 2>&1
rc=$?; tail -2 $O/maxf.log; [[ $rc -ne 0 ]] && { tail -30 $O/maxf.log; exit 1; }
timeout -k 10 900 bash scripts/r06_pmc.sh r06t > $O/pmc.log 2>&1; rc=$?; grep -v "^c[23] pass" $O/pmc.log | tail -40; exit $rc
