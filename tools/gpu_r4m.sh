#!/bin/bash
# round 4: per-step overhead floor of the N > 1 path (launches, flag waits):
# two gloo ranks sharing the GPU over P2P windows at small n, K = 1 / 2 / 4
# measured by the bench; then the world-1 native path at the same sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4m; mkdir -p $O
for n in 200000 1000000 2500000; do
  LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --n-rows $n --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/p2p_n$n.log 2>&1 || exit 1
  LHPC_DIST_NATIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 1 --n-rows $n --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/w1_n$n.log 2>&1 || exit 1
done
