#!/bin/bash
# Round-4 PMC of the map and partition (scripts/pmc_mappart.sh r04; HBM bytes for bench.py's
# roofline.traffic via pmc_summary.py --json), then the default bench line twice (box-to-box spread).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R
bash scripts/pmc_mappart.sh r04 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_r04 map_fused part_ --json gpurun_out/pmc_r04/summary.json || exit 1
cat gpurun_out/pmc_r04/summary.json
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/pmc_r04/bench$i.json 2> gpurun_out/pmc_r04/bench$i.err || { tail -20 gpurun_out/pmc_r04/bench$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'], d['roofline']['ms_per_launch'])" gpurun_out/pmc_r04/bench$i.json
done
