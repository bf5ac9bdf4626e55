#!/bin/bash
# r5 session AR: the driver's multi-GPU launch line rehearsed with ranks sharing the one GPU
# (MIINT_OVERSUBSCRIBE=1: RCCL over loopback sockets) at 2, 4 and 8 ranks, every extra on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
for n in 2 4 8; do
  MIINT_OVERSUBSCRIBE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/ar_torchrun_np$n.json 2> $O/ar_torchrun_np$n.err || { echo "np$n failed"; tail -30 $O/ar_torchrun_np$n.err; exit 1; }
done
echo "exit 0"
