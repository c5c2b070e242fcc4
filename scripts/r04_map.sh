#!/bin/bash
# Fused map phase stamps (probes library), the product library's map kernel time, and SQ PMC passes
# over the map kernel alone (scripts/map_once.py).  Every step time-limited; stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/${1:-map}; mkdir -p $O
cd $R
FASTKMER_LIB=$R/fastkmer_amd/lib_probes/libfastkmer.so FK_MAP_REPS=5 timeout -k 10 120 python -u scripts/map_cycles.py > $O/map_cycles.txt 2>&1 || { tail -20 $O/map_cycles.txt; exit 1; }
cat $O/map_cycles.txt
FK_MAP_REPS=9 timeout -k 10 120 python -u scripts/map_once.py > $O/map_once.txt 2>&1 || { tail $O/map_once.txt; exit 1; }
cat $O/map_once.txt
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  FK_MAP_REPS=3 timeout -s KILL 90 rocprofv3 --pmc $grp -d "$O/p$i" -o run --output-format csv -- python3 "$R/scripts/map_once.py" > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [[ $rc -ne 0 ]] && { tail -5 "$O/p$i.log"; exit $rc; }
done
python3 "$R/scripts/pmc_kernels.py" "$O" map_fused > $O/pmc_map.txt 2>&1; cat $O/pmc_map.txt
cd $R
if [ -n "$C3" ]; then
  timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }; cat $O/c3.json
  for pa in 2 3; do
    FASTKMER_PRECOUNT=1 FASTKMER_PRECOUNT_AT=$pa timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_pre$pa.json 2> $O/c3_pre$pa.err || { tail -20 $O/c3_pre$pa.err; exit 1; }; cat $O/c3_pre$pa.json
  done
fi
cd /tmp
FK_MAP_REPS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$O/p9" -o run --output-format csv -- python3 "$R/scripts/map_once.py" > "$O/p9.log" 2>&1 || { echo "icache pass rc=$?"; exit 0; }
python3 "$R/scripts/pmc_kernels.py" "$O" map_fused > $O/pmc_map.txt 2>&1; cat $O/pmc_map.txt
