#!/bin/bash
# round 4, last: bench.py's N>1 code paths on the final build — the native
# lhpc_dist_* path at world 1 over RCCL (C2, C3, CG) and two gloo ranks
# sharing the GPU over peer stores (C2); the real N = 2..8 runs are the driver's
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4final; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for wl in c2 c3 cg; do
  LHPC_DIST_NATIVE=1 timeout -k 10 400 $TR --nproc-per-node 1 --master-port 29581 bench.py --workload $wl \
    --steps 20 --warmup 3 --no-cpu-baseline > $O/native_world1_$wl.log 2>&1 || exit 1
done
LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 400 $TR --nproc-per-node 2 --master-port 29582 bench.py --gpus 2 \
  --steps 20 --warmup 3 --no-cpu-baseline > $O/p2p_gloo2_c2.log 2>&1 || exit 1
