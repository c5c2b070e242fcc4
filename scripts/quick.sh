#!/bin/bash
# GPU tests (FK_TESTS, default fused/parity/pieces; set it inside the gpurun command), the bench and
# a kernel-trace profile of the bench (gpurun_out/q_*): gpurun -- "FK_TESTS=... bash scripts/quick.sh"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
T=${FK_TESTS:-"tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_pieces.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/q_tests.log 2>&1 || { tail -30 $O/q_tests.log; exit 1; }
tail -2 $O/q_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/q_bench.json 2> $O/q_bench.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/q_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/q_prof.log 2>&1 || exit 1
