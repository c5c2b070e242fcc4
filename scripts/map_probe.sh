#!/bin/bash
# needs the probes library: python -m fastkmer_amd.build --probes (built here, travels with the tree)
# Fused map phases: full kernel, stop after byte classes + line state (probe 1), after compaction (probe 2)
for p in 0 1 2 3 4; do
  FASTKMER_LIB=$GRAFT_REPO_ROOT/fastkmer_amd/lib_probes/libfastkmer.so FASTKMER_FUSED_PROBE=$p FK_MAP_REPS=9 timeout -k 10 120 python -u scripts/map_once.py | sed "s/^/probe $p: /" || exit 1
done
