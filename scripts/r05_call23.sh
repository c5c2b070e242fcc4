#!/bin/bash
# Round 5 23rd GPU call: five / six staged pieces per job (-DFK_STAGE_MAXP, lib_maxp5 / lib_maxp6) with
# cuts that shrink toward the job's end, against the four-piece default; configs[1] and the
# configs[2] load, alternating; the pieces tests on lib_maxp5.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05w; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()}, round(d.get("pcie_h2d_GBps") or 0, 2))
PYEOF
}
L5=FASTKMER_LIB=$R/fastkmer_amd/lib_maxp5/libfastkmer.so
L6=FASTKMER_LIB=$R/fastkmer_amd/lib_maxp6/libfastkmer.so
for rep in 1 2; do
  run c3_default X=1 python -u bench.py --workload c3 $B || exit 1
  run c3_p5_0.4,0.65,0.82,0.93 $L5 FASTKMER_PIECE_CUTS=0.4,0.65,0.82,0.93 python -u bench.py --workload c3 $B || exit 1
  run c3_p5_0.4,0.7,0.88,0.96 $L5 FASTKMER_PIECE_CUTS=0.4,0.7,0.88,0.96 python -u bench.py --workload c3 $B || exit 1
  run c3_p6_0.35,0.6,0.78,0.9,0.96 $L6 FASTKMER_PIECE_CUTS=0.35,0.6,0.78,0.9,0.96 python -u bench.py --workload c3 $B || exit 1
  run c2_default X=1 python -u bench.py $B || exit 1
  run c2_p5_0.4,0.65,0.82,0.93 $L5 FASTKMER_PIECE_CUTS=0.4,0.65,0.82,0.93 python -u bench.py $B || exit 1
  run c2_p6_0.35,0.6,0.78,0.9,0.96 $L6 FASTKMER_PIECE_CUTS=0.35,0.6,0.78,0.9,0.96 python -u bench.py $B || exit 1
done
FASTKMER_LIB=$R/fastkmer_amd/lib_maxp5/libfastkmer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pieces.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_p5.log 2>&1
tail -3 $O/tests_p5.log; grep -E "FAILED|ERROR" $O/tests_p5.log | head
