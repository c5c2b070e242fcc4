#!/bin/bash
# one rocprofv3 PMC pass (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU,
# SQ_INSTS_VALU, ...) over the fused map kernel (scripts/map_once.py: the configs[1] input in HBM) and,
# with the same counters, over the VALU issue micro-benchmark (scripts/ubench/op_survey: 8 chains per
# wave, 8 waves per SIMD), so that cycles per wave64 VALU instruction per SIMD come from the GPU's own
# cycle counter (GRBM_GUI_ACTIVE / 8 XCDs) instead of a wall time at an assumed clock.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/valu; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$O/p1" -o run --output-format csv -- "$R/scripts/ubench/op_survey" > "$O/ubench.log" 2>&1 \
  || { echo "ubench pmc rc=$?"; tail -5 "$O/ubench.log"; exit 1; }
FK_MAP_REPS=3 timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$O/p2" -o run --output-format csv -- python3 "$R/scripts/map_once.py" > "$O/map.log" 2>&1 \
  || { echo "map pmc rc=$?"; tail -5 "$O/map.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/t" -o run --output-format csv -- python3 "$R/scripts/map_once.py" > "$O/map_trace.log" 2>&1 \
  || { echo "map trace rc=$?"; tail -5 "$O/map_trace.log"; exit 1; }
python3 "$R/scripts/valu_table.py" "$O" > "$O/valu_table.txt" 2>&1; cat "$O/valu_table.txt"
