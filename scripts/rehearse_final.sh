#!/bin/bash
# End-of-round rehearsals of the N > 1 path on one GPU: one rank's 6.25 GB configs[2] shard through
# the exchange path (device memory left), a 2-rank local rehearsal at 3 GB per rank, and the N = 1
# configs[2] line at its full 6.25 GB per GPU (host input; gpurun_out/rf_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash scripts/rehearse_c3_rank.sh || exit 1
timeout -k 10 400 python -u bench.py --rehearse-local 2 --bytes-per-gpu 3000000000 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/rf_local2.json 2> $O/rf_local2.err || { tail -20 $O/rf_local2.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/rf_c3_n1.json 2> $O/rf_c3_n1.err || { tail -20 $O/rf_c3_n1.err; exit 1; }
