#!/bin/bash
# Rehearsal of the driver's N > 1 bench launch on a one-GPU box: torchrun with 2 ranks sharing the
# GPU over gloo (records staged through host memory), default rounds and the size-aware placement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; tag=${1:-reh}
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-host-leg \
    > $OUT/${tag}_n2.json 2> $OUT/${tag}_n2.err
rc=$?; cut -c1-600 $OUT/${tag}_n2.json; [[ $rc -ne 0 ]] && { tail -20 $OUT/${tag}_n2.err; exit $rc; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-host-leg --balance \
    > $OUT/${tag}_n2b.json 2> $OUT/${tag}_n2b.err
rc=$?; cut -c1-300 $OUT/${tag}_n2b.json; [[ $rc -ne 0 ]] && { tail -20 $OUT/${tag}_n2b.err; exit $rc; }
exit 0
