#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for f2 in 7 8; do
  FASTKMER_F2=$f2 timeout -k 10 200 python3 -u scripts/probe_scale.py 8 | sed "s/^/F2=$f2 /" || exit 1
done
for f2 in 4 6; do
  FASTKMER_F2=$f2 timeout -k 10 200 python3 -u scripts/probe_scale.py 1 | sed "s/^/F2=$f2 /" || exit 1
done
