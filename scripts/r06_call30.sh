#!/bin/bash
# Round 6, 30th GPU call: the configs[2]-load tail with five staged pieces (kernel trace, one step after a
# warmup step): where the time after the last map launch goes now.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06ze; mkdir -p $O
cd $R
export TMPDIR=/tmp
for wl in c3 c2; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 $R/bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$wl.json 2> $O/prof_$wl.err) || { echo "prof $wl failed"; tail -5 $O/prof_$wl.err; exit 1; }
  python3 $R/scripts/kstats.py $O/prof_$wl/run_kernel_stats.csv 40 > $O/kstats_$wl.txt
  python3 $R/scripts/tail_timeline.py $O/prof_$wl/run_kernel_trace.csv > $O/tail_$wl.txt
  echo "== $wl"; tail -1 $O/tail_$wl.txt
done
