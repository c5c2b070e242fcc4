#!/bin/bash
# smoke (bit-exact vs the oracle), map A/B vs FK_MAPV=1, then the map stamps / PMC / configs[2] runs
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
bash scripts/ab_map.sh v1 || exit 1
C3=1 bash scripts/r04_map.sh map1
