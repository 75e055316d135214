#!/bin/bash
# Rehearsal of bench.py's N>1 path on a 1-GPU box: 2 ranks sharing cuda:0 over
# gloo (RCCL cannot put two ranks on one GPU).  Exercises the interleaved-block
# plans, the async all-gather overlap, DistCG's all-reduce/all-gather and the
# max-over-ranks timing with device tensors.  The real N=2..8 runs are the driver's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export LHPC_DIST_BACKEND=gloo
for WL in ${WLS:-c2 cg}; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --workload $WL --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearsal_$WL.log 2>&1 || exit 1
done
