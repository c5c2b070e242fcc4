#!/bin/bash
# rocprofv3 kernel stats of the bench for one workload: prof_workload.sh c3 [bytes]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
W=${1:-c2}; B=${2:-1000000000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pw_$W -o run -- python3 $R/bench.py --workload $W --bytes-per-gpu $B --steps 5 --warmup 1 --no-cpu-baseline > $O/pw_$W.json 2> $O/pw_$W.err || exit 1
