#!/bin/bash
# Round 6, 9th GPU call: the wave tiers' staged key addresses from one scalar base per row of 64 keys when
# the row lies in one piece, the 128-bit always-CAS dedupe as default; parity of the product library and of
# the 64-bit always-CAS variant (lib_w64cas, FK_W64_CAS=1); A/B lines against lib_base6 at configs[1] and
# the configs[2] / configs[3] loads; PMC of the 64-bit wave tier at the configs[2] load.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06i; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_pieces.py \
  tests/test_gpu_hash.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -gt 1 ]] && { echo "parity rc=$rc"; tail -30 $O/parity.log; exit 1; }
FASTKMER_LIB=$R/fastkmer_amd/lib_w64cas/libfastkmer.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_wave.py tests/test_gpu_pieces.py -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/parity_cas.log 2>&1
rc=$?; tail -2 $O/parity_cas.log; grep -E "FAILED|ERROR" $O/parity_cas.log | head -20
[[ $rc -gt 1 ]] && { echo "parity cas rc=$rc"; tail -30 $O/parity_cas.log; exit 1; }
B="--steps 5 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
OLD=FASTKMER_LIB=$R/fastkmer_amd/lib_base6/libfastkmer.so
CAS=FASTKMER_LIB=$R/fastkmer_amd/lib_w64cas/libfastkmer.so
for r in 1 2; do
  line c4_old$r c4 $OLD || exit 1
  line c4_new$r c4 X=1 || exit 1
  line c3_old$r c3 $OLD || exit 1
  line c3_new$r c3 X=1 || exit 1
  line c3_cas$r c3 $CAS || exit 1
  line c2_old$r c2 $OLD || exit 1
  line c2_new$r c2 X=1 || exit 1
  line c2_cas$r c2 $CAS || exit 1
done
export TMPDIR=/tmp
kst() {  # name, env assignments: kernel stats of one configs[2]-load job
  local name=$1; shift
  (cd /tmp && timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
    python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/prof_$name.json 2> $O/prof_$name.err) || { echo "prof $name failed"; tail -5 $O/prof_$name.err; return 1; }
  python3 $R/scripts/kstats.py $O/prof_$name/run_kernel_stats.csv 40 > $O/kstats_$name.txt
  echo "$name: $(grep -E 'count64_wave<2|count128_wave<2' $O/kstats_$name.txt | head -1)"
}
kst old $OLD || exit 1
kst new X=1 || exit 1
kst cas $CAS || exit 1
P=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR"; do
  P=$((P+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "count64_wave" -d $O/pmc$P -o run \
    --output-format csv -- python3 $R/bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline --no-device-leg \
    --c3-leg off > $O/pmc$P.log 2>&1) || { echo "pmc pass $P failed"; tail -5 $O/pmc$P.log; exit 1; }
done
python3 - $O <<'EOF'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fk::", "")[:60]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in acc.items():
    print(n)
    for k in sorted(c):
        print(f"  {k:24s} {c[k]:.4g}")
EOF
