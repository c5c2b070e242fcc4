#!/bin/bash
# Level-2 expansion workgroups sized to the keys per super-cell (staged pieces: 128 / 256 threads),
# every piece expanded in two levels: the piece / parity / configs / hash GPU tests, host-input
# bench A/B of FASTKMER_X2_L2 (0 = by keys per super-cell; 128 / 256 / 512 forced) at configs[1]
# and at the configs[3] shape (k = 55, workload c4), rocprof kernel stats of the default
# (gpurun_out/x2_*).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
    tests/test_gpu_hash.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/x2_tests.log 2>&1 \
    || { tail -40 $O/x2_tests.log; exit 1; }
tail -2 $O/x2_tests.log
bash scripts/ab_env.sh FASTKMER_X2_L2 "0 512 256 128" || exit 1
BENCH_ARGS="--workload c4" bash scripts/ab_env.sh FASTKMER_X2_L2 "0 512" || exit 1
cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/x2_prof -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/x2_prof.log 2>&1 || exit 1
