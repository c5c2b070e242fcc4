#!/bin/bash
# PMC passes over the map and partition kernels (scripts/count_once.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_${1:-mp}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export FK_HT=0
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT TCC_MISS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/scripts/count_once.py" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
done
python3 "$ROOT/scripts/pmc_kernels.py" "$OUT" part_ map_fused
