#!/bin/bash
# Round 6, 23rd GPU call: the mid wave tier launched before the split on the side stream (lib_prev = queued
# after the split's read-back): tier / heavy-bucket parity, A/B lines at configs[1] and the configs[2] /
# configs[3] loads, the configs[1] tail; then PMC of the wave tiers on the final tree (configs[2] load: 64-bit,
# configs[3] load: 128-bit) for the SALU / VALU / bank-conflict figures.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06w; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pieces.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -ne 0 ]] && { echo "parity rc=$rc"; grep -E "^E " $O/parity.log | head -30; exit 1; }
B="--steps 6 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
PV=FASTKMER_LIB=$R/fastkmer_amd/lib_prev/libfastkmer.so
for r in 1 2 3; do
  line c2_new$r c2 X=1 || exit 1
  line c2_prev$r c2 $PV || exit 1
done
for r in 1 2; do
  line c4_new$r c4 X=1 || exit 1
  line c4_prev$r c4 $PV || exit 1
  line c3_new$r c3 X=1 || exit 1
  line c3_prev$r c3 $PV || exit 1
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c2 -o run -- python3 $R/bench.py \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off > $O/trace_c2.json 2> $O/trace_c2.err) || { echo "trace failed"; exit 1; }
python3 $R/scripts/tail_timeline.py $O/trace_c2/run_kernel_trace.csv > $O/tail_c2.txt; tail -1 $O/tail_c2.txt
P=0
for wl in c3 c4; do
  RX=count64_wave; [[ $wl == c4 ]] && RX=count128_wave
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
