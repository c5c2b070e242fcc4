#!/bin/bash
# useHT combine kernel stopped after each phase (FASTKMER_LH_PROBE): 1 expansion, 2 inserts, 0 all
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for p in 1 2 0; do
  FK_HT=1 FASTKMER_LH_PROBE=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/lhp$p -o run --output-format csv \
      -- python3 $ROOT/scripts/count_once.py > $OUT/lhp$p.log 2>&1 || exit 1
  echo "probe $p: $(grep k_ht_combine $OUT/lhp$p/run_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
