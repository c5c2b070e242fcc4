#!/bin/bash
# Round 6, 36th GPU call: the heavy tiers' cost per key against the wave tier's, each kernel alone (lib_noside:
# -DFK_TIER_SIDE=0, the heavy tiers after the wave tier on one stream): the configs[2] and configs[3] loads
# counted whole from HBM (scripts/count_once.py, two jobs), kernel stats of each.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zl; mkdir -p $O
cd $R
export TMPDIR=/tmp
NS=$R/fastkmer_amd/lib_noside/libfastkmer.so
for wl in c3 c4; do
  if [ $wl = c3 ]; then K=28; M=10; RL=100; else K=55; M=12; RL=150; fi
  (cd /tmp && timeout -k 10 300 env FASTKMER_LIB=$NS FK_B=8192 FK_BYTES=6250000000 FK_GENOME=3000000000 FK_JOBS=2 \
    FK_K=$K FK_M=$M FK_RL=$RL rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 $R/scripts/count_once.py > $O/prof_$wl.log 2>&1) || { echo "prof $wl failed"; tail -5 $O/prof_$wl.log; exit 1; }
  python3 $R/scripts/kstats.py $O/prof_$wl/run_kernel_stats.csv 30 > $O/kstats_$wl.txt
  echo "== $wl"; tail -2 $O/prof_$wl.log; head -14 $O/kstats_$wl.txt
done
