#!/bin/bash
# Round 6, 14th GPU call: where each staged piece's work falls against the landing input at the configs[2]
# load, for the default piece cuts and for later ones (job_pieces.py over a rocprofv3 kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06n; mkdir -p $O
cd $R
export TMPDIR=/tmp
tr() {  # name, then env assignments
  local name=$1; shift
  (cd /tmp && timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --output-format csv -d $O/trace_$name -o run -- \
    python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off \
    > $O/trace_$name.json 2> $O/trace_$name.err) || { echo "trace $name failed"; tail -5 $O/trace_$name.err; return 1; }
  python3 $R/scripts/job_pieces.py $O/trace_$name/run_kernel_trace.csv 0.4 > $O/pieces_$name.txt
  echo "== $name"; cat $O/pieces_$name.txt
}
tr default X=1 || exit 1
tr late FASTKMER_PIECE_CUTS=0.6,0.82,0.94 || exit 1
