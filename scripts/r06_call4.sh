#!/bin/bash
# Round 6, 4th GPU call: RCCL bounded waits (kernel staging copies); parity of the 128-bit fingerprint tier (LDS
# exact fallback) and of the 64-bit fingerprint variant (lib_w64fp768); A/B of the 64-bit fingerprint tables
# (768 / 1024 slots) at configs[1] and the configs[2] load; the configs[3] line; piece-cut A/B at configs[2].
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06d; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -k "rccl" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/comm.log 2>&1
rc=$?; tail -3 $O/comm.log; grep -E "FAILED|ERROR|^E " $O/comm.log | head -20
[[ $rc -gt 1 ]] && { echo "comm rc=$rc"; tail -30 $O/comm.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave.py -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; grep -E "FAILED|ERROR" $O/parity.log | head -20
[[ $rc -gt 1 ]] && { echo "parity rc=$rc"; tail -30 $O/parity.log; exit 1; }
FASTKMER_LIB=$R/fastkmer_amd/lib_w64fp768/libfastkmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_wave.py tests/test_gpu_pieces.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity_fp768.log 2>&1
rc=$?; tail -2 $O/parity_fp768.log; grep -E "FAILED|ERROR" $O/parity_fp768.log | head -20
[[ $rc -gt 1 ]] && { echo "parity fp768 rc=$rc"; tail -30 $O/parity_fp768.log; exit 1; }
B="--steps 6 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
L768=FASTKMER_LIB=$R/fastkmer_amd/lib_w64fp768/libfastkmer.so
L1024=FASTKMER_LIB=$R/fastkmer_amd/lib_w64fp1024/libfastkmer.so
for r in 1 2; do
  line c3_base$r c3 X=1 || exit 1
  line c3_fp768_$r c3 $L768 || exit 1
  line c3_fp1024_$r c3 $L1024 || exit 1
  line c2_base$r c2 X=1 || exit 1
  line c2_fp768_$r c2 $L768 || exit 1
done
line c4 c4 X=1 || exit 1
for cuts in 0.6,0.82,0.94 0.55,0.78,0.93 0.65,0.85,0.95; do
  line c3_cuts_$cuts c3 FASTKMER_PIECE_CUTS=$cuts || exit 1
  line c2_cuts_$cuts c2 FASTKMER_PIECE_CUTS=$cuts || exit 1
done
line c3_base3 c3 X=1 || exit 1
line c2_base3 c2 X=1 || exit 1
