#!/bin/bash
# mid wave tier: its parity tests, configs[2] per-GPU bench with / without it; map phase stamps
# (per-wave accumulation); then the full GPU suite.  Each step time-limited; stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "mid_tier or big_bins or max_fine or count_variants" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/mid_tests.log 2>&1 || { tail -40 $O/mid_tests.log; exit 1; }
tail -3 $O/mid_tests.log
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
for mt in 1 0; do
  FASTKMER_MID_TIER=$mt timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_mid$mt.json 2> $O/c3_mid$mt.err || { tail -20 $O/c3_mid$mt.err; exit 1; }
  cat $O/c3_mid$mt.json
done
O=gpurun_out bash scripts/r04_suite.sh
