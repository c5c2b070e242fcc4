#!/bin/bash
# PMC passes over the configs[2]-load sorted count (6.25 GB, 3 Gbp genome, B = 8192; scripts/count_once.py):
# the bucket tiers -- VALU / LDS instructions, LDS bank-conflict cycles, HBM bytes per launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_${1:-wave}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export FK_HT=0 FK_BYTES=6250000000 FK_GENOME=3000000000 FK_B=8192
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT TCC_MISS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/scripts/count_once.py" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [[ $rc -ne 0 ]] && exit $rc
done
python3 "$ROOT/scripts/pmc_kernels.py" "$OUT" count64 split64 join expand_sc fine_sc hist_bin > "$OUT/summary.txt"
cat "$OUT/summary.txt"
