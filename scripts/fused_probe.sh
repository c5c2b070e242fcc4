#!/bin/bash
# needs the probes library: python -m fastkmer_amd.build --probes (built here, travels with the tree)
# Fused map kernel stopped after each phase (FASTKMER_FUSED_PROBE): 1 byte classes + line state,
# 2 compaction, 3 signature passes, 4 look-back, 0 whole kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for p in 1 2 3 4 0; do
  echo -n "probe $p: "
  FASTKMER_LIB=$GRAFT_REPO_ROOT/fastkmer_amd/lib_probes/libfastkmer.so FASTKMER_FUSED_PROBE=$p FK_MAP_REPS=15 timeout -k 10 120 python3 scripts/map_once.py || exit 1
done
