#!/bin/bash
# Exchange-path staging at the job's cuts: comm / pieces / hash GPU tests, then configs[2] per-GPU load
# through the exchange path with one in-process rank (host trace), and two ranks at 1 GB each.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/xch2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_comm.py tests/test_gpu_pieces.py tests/test_gpu_hash.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
FASTKMER_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --rehearse-local 1 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl1.json 2> $O/rl1.err || { tail -20 $O/rl1.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rl1 c3', round(d['ms_per_step'],2), d['stages_ms'])" $O/rl1.json
grep htrace $O/rl1.err | tail -8
timeout -k 10 300 python -u bench.py --rehearse-local 2 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl2.json 2> $O/rl2.err || { tail -20 $O/rl2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rl2 c1', round(d['ms_per_step'],2), d['stages_ms'])" $O/rl2.json
