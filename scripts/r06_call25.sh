#!/bin/bash
# Round 6, 25th GPU call: the 1024-key mid wave tier on a stream of its own beside the wave tier and the split
# chain (FK_MID_SIDE default; lib_nomidside = on the split's stream after it): parity, A/B lines at configs[1]
# (where the mid tier ended after the wave tier) and the configs[3] load (128-bit mid tier), configs[1] tail.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06y; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_write.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -ne 0 ]] && { echo "parity rc=$rc"; grep -E "^E " $O/parity.log | head -30; exit 1; }
B="--steps 6 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
NM=FASTKMER_LIB=$R/fastkmer_amd/lib_nomidside/libfastkmer.so
for r in 1 2 3; do
  line c2_ms$r c2 X=1 || exit 1
  line c2_noms$r c2 $NM || exit 1
done
for r in 1 2; do
  line c4_ms$r c4 X=1 || exit 1
  line c4_noms$r c4 $NM || exit 1
done
line c3_ms c3 X=1 || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c2 -o run -- python3 $R/bench.py \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off > $O/trace_c2.json 2> $O/trace_c2.err) || { echo "trace failed"; exit 1; }
python3 $R/scripts/tail_timeline.py $O/trace_c2/run_kernel_trace.csv > $O/tail_c2.txt; tail -1 $O/tail_c2.txt
