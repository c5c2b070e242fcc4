#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Each step has
# its own time limit and the script stops at the first failure.
# Usage: bash scripts/gpu_check.sh [tests|bench|prof|all] [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
what=${1:-all}
tag=${2:-run}
if [[ $what == tests || $what == all ]]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider --tb=short -rf \
      > "$OUT/gpu_tests_$tag.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests_$tag.log"; [[ $rc -ne 0 ]] && { echo "tests rc=$rc"; exit $rc; }
fi
if [[ $what == bench || $what == all ]]; then
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > "$OUT/bench_$tag.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_$tag.log"; [[ $rc -ne 0 ]] && { echo "bench rc=$rc"; exit $rc; }
fi
if [[ $what == prof || $what == all ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_$tag.log" 2>&1
  rc=$?; echo "prof rc=$rc"; exit $rc
fi
