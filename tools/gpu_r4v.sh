#!/bin/bash
# round 4: bench.py --workload c5 --gpus N with the P2P halo, rehearsed as
# gloo ranks sharing the GPU (2 and 3 ranks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4v; mkdir -p $O
for w in 2 3; do
  LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w \
    --master-addr 127.0.0.1 --master-port 2958$w bench.py --gpus $w --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/c5_w$w.log 2>&1 || exit 1
done
