#!/bin/bash
# One rank's configs[2] shard (6.25 GB, the 50 GB job over 8 GPUs) through the exchange path with an
# in-process communicator of one rank: step time and the device memory left (FASTKMER_BENCH_MEMINFO)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
FASTKMER_BENCH_MEMINFO=1 timeout -k 10 600 python -u bench.py --rehearse-local 1 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-device-leg > $O/rl1c3.json 2> $O/rl1c3.err || { tail -20 $O/rl1c3.err; exit 1; }
grep meminfo $O/rl1c3.err
