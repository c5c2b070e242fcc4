#!/bin/bash
# configs[1] host-input tail: staged cut sets A/B (alternated), host timestamps of one step, and the
# kernel + copy timeline of the default step.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/tail; mkdir -p $O
for r in 1 2; do
  for cuts in default 0.5,0.8,0.95 0.55,0.85,0.95 0.4,0.7,0.9; do
    if [ $cuts = default ]; then unset FASTKMER_PIECE_CUTS; else export FASTKMER_PIECE_CUTS=$cuts; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-device-leg > $O/b_$cuts.$r.json 2>> $O/b.err || { tail $O/b.err; exit 1; }
    echo "cuts $cuts run $r: $(python3 -c "import json; d=json.load(open('$O/b_$cuts.$r.json')); print(round(d['ms_per_step'],2), round(d['value']/1e9,2))")"
  done
done
unset FASTKMER_PIECE_CUTS
FASTKMER_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/ht.json 2> $O/ht.err || exit 1
tail -40 $O/ht.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg > $O/tl.log 2>&1 || exit 1
DB=$(find $O/tl -name "*.db" -print -quit); python3 $R/scripts/timeline.py "$DB" 30 > $O/timeline.txt 2>&1; tail -70 $O/timeline.txt
