#!/bin/bash
# configs[2] per-GPU load through the exchange path with one in-process rank (--rehearse-local 1): host
# timestamps of the tail (FASTKMER_HOST_TRACE) and the kernel + copy timeline of one step, against N=1.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/xtail; mkdir -p $O
FASTKMER_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --rehearse-local 1 --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl1.json 2> $O/rl1.err || { tail -20 $O/rl1.err; exit 1; }
FASTKMER_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/n1.json 2> $O/n1.err || { tail -20 $O/n1.err; exit 1; }
grep -c . $O/rl1.err $O/n1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl -o run -- python3 $R/bench.py --rehearse-local 1 --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
DB=$(find $O/tl -name "*.db" -print -quit); python3 $R/scripts/timeline.py "$DB" 60 > $O/timeline.txt 2>&1; tail -80 $O/timeline.txt
