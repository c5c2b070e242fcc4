#!/bin/bash
# Round 6 PMC (separate passes, no trace domains): HBM bytes, VALU and LDS counters per kernel of
#   c2: configs[1]'s 1 GB job counted whole from HBM (scripts/count_once.py: 3 jobs), as round 4's table;
#   c3: configs[2]'s per-GPU load (6.25 GB, B = 8192, 3 Gbp genome; 1 job: the split's copy included).
# Usage: bash scripts/r06_pmc.sh TAG
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_ACTIVE_INST_VALU"
         "FETCH_SIZE" "WRITE_SIZE")
for wl in c2 c3; do
  OUT=$R/gpurun_out/pmc_${TAG}_$wl; mkdir -p "$OUT"
  if [[ $wl == c3 ]]; then export FK_BYTES=6250000000 FK_GENOME=3000000000 FK_B=8192 FK_JOBS=1; JOBS=1; FB=6249999954
  else export FK_BYTES=1000000000 FK_GENOME=100000000 FK_B=2048 FK_JOBS=3; JOBS=3; FB=999999906; fi
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/scripts/count_once.py" > "$OUT/p$i.log" 2>&1
    rc=$?; echo "$wl pass $i rc=$rc $(tail -1 $OUT/p$i.log)"; [[ $rc -ne 0 ]] && exit $rc
  done
  python3 "$R/scripts/pmc_table.py" "$OUT" $FB $JOBS --json "$OUT/summary.json" > "$OUT/table.txt" || exit 1
  cat "$OUT/table.txt"
done
