#!/bin/bash
# Count stage vs the super-cell split FASTKMER_F2 (cells per super-cell = 2^F2) at configs[1] and the
# configs[2] shape: gpurun_out/f2.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for g in 100000000 3000000000; do
for f2 in -1 4 6 7; do
  if [ $f2 = -1 ]; then unset FASTKMER_F2; else export FASTKMER_F2=$f2; fi
  B=2048; [ $g = 3000000000 ] && B=8192
  FK_B=$B FK_GENOME=$g timeout -k 10 200 python -u scripts/count_once.py 2>/dev/null | sed "s/^/genome $g F2 $f2: /" | tee -a $O/f2.log || exit 1
done
done
