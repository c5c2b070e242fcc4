#!/bin/bash
# SQ counters of the split map's two kernels (parse: MODE 1, passes: MODE 2) and of the fused kernel
# (FASTKMER_SPLIT_MAP=0): VALU / SALU / LDS instructions, wave cycles, busy cycles.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/pmcs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for sp in 1 0; do
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  FASTKMER_SPLIT_MAP=$sp FK_MAP_REPS=3 timeout -s KILL 90 rocprofv3 --pmc $grp -d "$O/p$i" -o run --output-format csv -- python3 "$R/scripts/map_once.py" > "$O/p$i.log" 2>&1
  rc=$?; echo "split=$sp pass $i rc=$rc"; [[ $rc -ne 0 ]] && { tail -5 "$O/p$i.log"; exit $rc; }
done
done
python3 "$R/scripts/pmc_kernels.py" "$O" map_fused > $O/pmc.txt 2>&1; cat $O/pmc.txt
