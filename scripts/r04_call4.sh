#!/bin/bash
# barrier-light parse (FK_MAPV 3) and the 6144-slot big tier: fused-map and tier parity tests, smoke,
# map A/B vs FK_MAPV 2 / 1, phase stamps; configs[2] per-GPU bench under rocprofv3 kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -v -k "block_and_big or parse_line" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash scripts/ab_map.sh v2 v1 || exit 1
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c3p -o run -- python3 $R/bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/c3p.log 2>&1 || { tail -20 $R/$O/c3p.log; exit 1; }
grep metric $R/$O/c3p.log
python3 $R/scripts/kstats.py $R/$O/c3p/run_kernel_stats.csv 14 > $R/$O/c3p_stats.txt; cat $R/$O/c3p_stats.txt
