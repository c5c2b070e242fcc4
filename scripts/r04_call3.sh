#!/bin/bash
# empty-bucket fix and mid tier: the failing random case + mid tests; map stamps with the load wait
# split out; configs[2] per-GPU bench under rocprofv3 kernel stats; then the full GPU suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "random_vs_oracle or mid_tier" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c3p -o run -- python3 $R/bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/c3p.log 2>&1 || { tail -20 $R/$O/c3p.log; exit 1; }
grep metric $R/$O/c3p.log
python3 $R/scripts/kstats.py $R/$O/c3p/run_kernel_stats.csv 30 > $R/$O/c3p_stats.txt; cat $R/$O/c3p_stats.txt
cd $R
bash scripts/r04_suite.sh
