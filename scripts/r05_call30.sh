#!/bin/bash
# Round 5 30th GPU call: configs[1] through the exchange path with one in-process rank -- kernel trace
# of its tail after the last byte, beside the local line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05zd; mkdir -p $O
cd $R
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
run c2 X=1 python -u bench.py $B || exit 1
run c2_x1 X=1 python -u bench.py --rehearse-local 1 $B || exit 1
run c2_x1_host FASTKMER_HOST_TRACE=1 python -u bench.py --rehearse-local 1 --steps 2 --warmup 1 --no-cpu-baseline --no-device-leg || exit 1
grep -c "" $O/c2_x1_host.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x1 -o run -- python3 $R/bench.py \
  --rehearse-local 1 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_x1.json 2> $O/prof_x1.err || { echo "prof failed"; tail -20 $O/prof_x1.err; exit 1; }
python3 $R/scripts/tail_timeline.py $O/prof_x1/run_kernel_trace.csv > $O/x1_c2_tail.txt && tail -1 $O/x1_c2_tail.txt
cd $R
python3 -c "import bench, os; n = bench.pin_to_gpu_numa(0); print('numa node of GPU 0:', n, 'cpus now', len(os.sched_getaffinity(0)))"
