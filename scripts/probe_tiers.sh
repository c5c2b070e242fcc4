#!/bin/bash
# count kernels at configs[1] under several env settings ("A=1,B=2" per argument; "-" = defaults),
# kernel stats per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/tiers_${1:-t}; mkdir -p "$OUT"; shift
cd /tmp && export TMPDIR=/tmp
i=0
for st in "$@"; do
  i=$((i+1))
  envs=(); [[ "$st" != "-" ]] && IFS=, read -ra envs <<< "$st"
  ( for e in "${envs[@]}"; do export "$e"; done
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/s$i" -o run --output-format csv \
      -- python3 -u "$ROOT/scripts/count_once.py" > "$OUT/s$i.log" 2>&1 )
  rc=$?; echo "[$st] rc=$rc $(grep '^count' "$OUT/s$i.log")"; [[ $rc -ne 0 ]] && exit $rc
  python3 - "$OUT/s$i/run_kernel_stats.csv" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:12]:
    if 'synth' in x['Name'] or 'map_fused' in x['Name'] or 'part_hist' in x['Name']: continue
    print(f"   {x['Name'][:58]:58s} calls={x['Calls']:>4} avg_ms={float(x['AverageNs'])/1e6:.3f}")
PY
done
