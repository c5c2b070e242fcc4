#!/bin/bash
# Round 5 32nd GPU call: exchange steps of at least 64 MB (a 1 GB job in ten steps) vs 128 MB (seven,
# lib_xmin128): comm tests, then configs[1] and the configs[2] load through the exchange path with one
# in-process rank, alternating.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05zf; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_comm.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR|Error" $O/tests.log | head -20
[[ $rc -ne 0 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
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
for v in default xmin128 default xmin128; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_x1_$v $L python -u bench.py --rehearse-local 1 $B || exit 1
  run c3_x1_$v $L python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
done
