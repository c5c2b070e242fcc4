#!/bin/bash
# Map-kernel A/B: scripts/map_once.py (HIP-event medians of 9 launches over the bench's 1 GB input)
# with the product library and with each variant library named on the command line
# (fastkmer_amd/lib_<name>/libfastkmer.so), alternated twice.  Every run time-limited.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/ab_map; mkdir -p $O
cd $R
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset FASTKMER_LIB; else export FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so; fi
    FK_MAP_REPS=9 timeout -k 10 120 python -u scripts/map_once.py > $O/$v.$r.txt 2>&1 || { tail $O/$v.$r.txt; exit 1; }
    echo "$v run $r: $(cat $O/$v.$r.txt)"
  done
done
unset FASTKMER_LIB
