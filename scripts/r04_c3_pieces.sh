#!/bin/bash
# configs[2] per-GPU load (6.25 GB, N = 1): staged pieces (default) against count + merge per piece
# (FASTKMER_PIECE_MODE=0) with fixed piece sizes: the GPU idles through most of the 113 ms of H2D, so
# pieces counted while the rest lands may pay although their distinct keys are counted again.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/c3p; mkdir -p $O
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$n.json $n
}
run staged FK_X=0 || exit 1
run merge_1g FASTKMER_PIECE_MODE=0 FASTKMER_PIECE_BYTES=1000000000 || exit 1
run merge_1.6g FASTKMER_PIECE_MODE=0 FASTKMER_PIECE_BYTES=1600000000 || exit 1
run merge_2.2g FASTKMER_PIECE_MODE=0 FASTKMER_PIECE_BYTES=2200000000 || exit 1
