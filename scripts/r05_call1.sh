#!/bin/bash
# Round 5 first GPU calls: the full GPU suite + smoke, the default bench line (N = 1 + the configs[2]-
# per-GPU leg), --gpus 2 on a one-GPU box (must fail loudly), the one-rank exchange rehearsal of
# configs[3] at its 6.25 GB per-GPU load with the memory left, and the VALU issue counter table.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05a; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 400 --timeout-method thread \
  -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[[ $rc -gt 1 ]] && { echo "suite rc=$rc"; tail -30 $O/suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
(timeout -k 10 120 python -u bench.py --gpus 2 --steps 1; echo "exit $?") > $O/gpus2.log 2>&1
cat $O/gpus2.log
FASTKMER_BENCH_MEMINFO=1 timeout -k 10 240 python -u bench.py --rehearse-local 1 --workload c4 --steps 5 --warmup 2 \
  > $O/rehearse1_c4.json 2> $O/rehearse1_c4.err || { tail -20 $O/rehearse1_c4.err; exit 1; }
cat $O/rehearse1_c4.json; grep meminfo $O/rehearse1_c4.err
bash scripts/r05_valu_pmc.sh || exit 1
