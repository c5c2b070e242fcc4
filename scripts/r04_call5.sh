#!/bin/bash
# coalesced tile loads (FK_MAPV 4): fused-map parity, smoke, map A/B vs FK_MAPV 3 / 1, stamps;
# configs[2] per-GPU bench with the last staged piece at 5 % (cuts 0.5, 0.8, 0.95) vs the default.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -v -k "fused or golden or baseline_c1 or two_word or parse_line or full_size" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash scripts/ab_map.sh v3 v1 || exit 1
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
for cuts in default 0.5,0.8,0.95; do
  if [ $cuts = default ]; then unset FASTKMER_PIECE_CUTS; else export FASTKMER_PIECE_CUTS=$cuts; fi
  timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_$cuts.json 2> $O/c3_$cuts.err || { tail -20 $O/c3_$cuts.err; exit 1; }
  echo "cuts $cuts: $(cat $O/c3_$cuts.json)"
done
unset FASTKMER_PIECE_CUTS
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
