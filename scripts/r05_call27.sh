#!/bin/bash
# Round 5 27th GPU call: exchange-path cuts 0.35/0.65/0.84 by default, H2D segments of a sixteenth of
# the call.  Pieces / comm / write tests; the exchange cuts around the new default; configs[1] through
# the exchange path (one and two in-process ranks) beside the local line; the configs[2] load.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05za; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_comm.py tests/test_gpu_write.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
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
for rep in 1 2; do
  run x1_default X=1 python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
  run x1_0.3,0.6,0.8 FASTKMER_PIECE_CUTS=0.3,0.6,0.8 python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
  run x1_0.33,0.62,0.82 FASTKMER_PIECE_CUTS=0.33,0.62,0.82 python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
  run c3 X=1 python -u bench.py --workload c3 $B || exit 1
  run c2 X=1 python -u bench.py $B || exit 1
  run c2_x1 X=1 python -u bench.py --rehearse-local 1 $B || exit 1
  run c2_x2 X=1 python -u bench.py --rehearse-local 2 $B || exit 1
done
