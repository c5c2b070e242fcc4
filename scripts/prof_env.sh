#!/bin/bash
# rocprofv3 kernel stats of the default bench under each value of one knob: prof_env.sh VAR "v1 v2"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
VAR=$1; VALS=$2
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pe_$v -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pe_$v.json 2> $O/pe_$v.err || exit 1
done
