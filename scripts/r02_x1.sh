#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
VARIANTS="- FASTKMER_X2_L1=512" bash scripts/r02_sort.sh x1 || exit 1
timeout -k 10 200 python3 -u scripts/probe_scale.py 8 || exit 1
FASTKMER_X2_L1=512 timeout -k 10 200 python3 -u scripts/probe_scale.py 8 || exit 1
