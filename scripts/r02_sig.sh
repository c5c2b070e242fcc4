#!/bin/bash
# GPU run for the bin-signature diagnostics: its tests, the
# distributed job test and a kernel-trace profile of the 1 GB test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
[ "${SIG_TESTS:-1}" = 0 ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
    tests/test_gpu_signatures.py "tests/test_distributed.py::test_find_bin_signatures_job_distributed" \
    > gpurun_out/sig_tests.log 2>&1 || { tail -40 gpurun_out/sig_tests.log; exit 1; }
[ "${SIG_TESTS:-1}" = 0 ] || { tail -5 gpurun_out/sig_tests.log; grep "bin signatures, 1 GB" gpurun_out/sig_tests.log; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sigprof -o sig --output-format csv -- \
    python -u -m pytest -x -q --timeout 240 --timeout-method thread -s \
    "tests/test_gpu_signatures.py::test_configs1_scale_linearity_and_rate" > gpurun_out/sig_prof.log 2>&1 \
    || { tail -30 gpurun_out/sig_prof.log; exit 1; }
grep "bin signatures, 1 GB" gpurun_out/sig_prof.log
find gpurun_out/sigprof -name "*kernel_stats.csv"
