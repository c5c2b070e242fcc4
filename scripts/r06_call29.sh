#!/bin/bash
# (second run, r06zd: the GPU files from test_gpu_pieces.py on -- r06zc stopped there on a test whose last cut fell under 128 MB)
# Round 6, 29th GPU call: five staged pieces for 64-bit jobs of >= 4 GB with the 128-bit kernels' piece
# loops kept at four (stage_npc<KW>): the whole GPU suite, then A/B lines against lib_p4 (FK_STAGE_MAXP=4,
# the round-6 4-piece schedule) at the configs[2] / configs[3] loads and configs[1], interleaved.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06zd; mkdir -p $O
cd $R
timeout -k 10 480 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_signatures.py tests/test_gpu_wave.py tests/test_gpu_write.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[[ $rc -ne 0 ]] && { echo "gpu tests rc=$rc"; tail -30 $O/gpu_tests.log; exit 1; }
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg --c3-leg off"
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P4=FASTKMER_LIB=$R/fastkmer_amd/lib_p4/libfastkmer.so
for r in 1 2 3; do
  line c3_p5_$r c3 X=1 || exit 1
  line c3_p4_$r c3 $P4 || exit 1
done
for r in 1 2; do
  line c2_p5_$r c2 X=1 || exit 1
  line c2_p4_$r c2 $P4 || exit 1
  line c4_p5_$r c4 X=1 || exit 1
  line c4_p4_$r c4 $P4 || exit 1
done
