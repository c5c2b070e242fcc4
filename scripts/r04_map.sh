#!/bin/bash
# Fused map phase stamps (probes library) and PMC of the product library's map kernel.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out; mkdir -p $O
cd $R
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
FK_MAP_REPS=9 timeout -k 10 120 python -u scripts/map_once.py > $O/map_once.txt 2>&1 || { tail $O/map_once.txt; exit 1; }
cat $O/map_once.txt
