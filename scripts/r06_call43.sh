#!/bin/bash
# Round 6, 43rd GPU call: PMC of the wave tiers and the heavy tiers on the final tree (configs[2] load: k_bucket_count64_wave, the key-range
# mid tier, the split, the in-order sub-buckets; configs[3] load: k_bucket_count128_wave), per launch, against r06w (profiles/r06w_pmc_wave_tiers.txt).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zs; mkdir -p $O
cd $R
export TMPDIR=/tmp
P=0
for wl in c3 c4; do
  RX="count64_wave|count64_parts|split64|sub_count64"; [[ $wl == c4 ]] && RX=count128_wave
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"; do
    P=$((P+1))
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$RX" -d $O/pmc$P -o run \
      --output-format csv -- python3 $R/bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-device-leg \
      --c3-leg off > $O/pmc$P.log 2>&1) || { echo "pmc pass $P failed"; tail -5 $O/pmc$P.log; exit 1; }
  done
done
python3 - $O <<'PYEOF'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fk::", "")[:62]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in acc.items():
    print(n)
    for k in sorted(c):
        print(f"  {k:24s} {c[k]:.4g}")
PYEOF
