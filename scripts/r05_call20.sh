#!/bin/bash
# Round 5 20th GPU call: H2D segments of 4 x 32 MB up to the ingest call's last tenth (32 MB there)
# -- pieces / comm / write tests, then configs[1] / configs[2] load A/B against one segment size
# (lib_seg1), alternating.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05t; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_comm.py tests/test_gpu_write.py \
  -m gpu -v --maxfail 3 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[[ $rc -gt 1 ]] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
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
for v in default seg1 default seg1; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_$v $L python -u bench.py $B || exit 1
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
done
run c3_rehearse1 X=1 python -u bench.py --workload c3 --rehearse-local 1 $B || exit 1
