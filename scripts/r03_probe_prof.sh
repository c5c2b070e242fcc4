#!/bin/bash
# pieces_probe under rocprofv3 kernel stats: where the per-piece counts and the merge spend their time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_pieces
FASTKMER_PIECE_BYTES=536870912 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pieces -o run --output-format csv -- python -u scripts/pieces_probe.py 512 > gpurun_out/prof_pieces.log 2>&1 || { tail -20 gpurun_out/prof_pieces.log; exit 1; }
find gpurun_out/prof_pieces -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/pieces_kernel_stats.csv
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/pieces_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  {int(r["Calls"]):6d}  {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
