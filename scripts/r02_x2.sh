#!/bin/bash
# level-1 kernel choice at the 4- and 8-GPU per-GPU bin sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in 4 8; do
  for v in 512 1024; do
    FASTKMER_X2_L1=$v timeout -k 10 200 python3 -u scripts/probe_scale.py $n | sed "s/^/L1=$v /" || exit 1
  done
done
timeout -k 10 200 python3 -u scripts/probe_scale.py 8 | sed "s/^/auto /" || exit 1
