#!/bin/bash
# Round 5 17th GPU call: mid wave tier tables of 1280 slots (lib_mid1280, 14.5 KB per wave) vs 1536.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r05q; mkdir -p $O
cd $R
B="--steps 8 --warmup 2 --no-cpu-baseline --no-device-leg"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python - "$O/$name.json" "$name" <<'PYEOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), {k: round(v, 2) for k, v in d["stages_ms"].items()})
PYEOF
}
for v in default mid1280 default mid1280; do
  L=X=1; [[ $v != default ]] && L=FASTKMER_LIB=$R/fastkmer_amd/lib_$v/libfastkmer.so
  run c2_$v $L python -u bench.py $B || exit 1
  run c3_$v $L python -u bench.py --workload c3 $B || exit 1
done
cd /tmp && export TMPDIR=/tmp
export FASTKMER_LIB=$R/fastkmer_amd/lib_mid1280/libfastkmer.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -20 $O/prof_c3.err; exit 1; }
python3 $R/scripts/kstats.py $O/prof_c3/run_kernel_stats.csv 14 | grep -E "1024u|split|sub_count|join"
