#!/bin/bash
# round 4: bench.py's native N > 1 path with the measured chunk count
# (K = 1, 2, 4): two gloo ranks sharing the GPU over P2P windows, then the
# world-1 RCCL form (LHPC_DIST_NATIVE=1).  Output under gpurun_out/r4i/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4i; mkdir -p $O
LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/rehearsal_p2p_c2.log 2>&1 || exit 1
LHPC_DIST_NATIVE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/native_world1_c2.log 2>&1 || exit 1
LHPC_DIST_NATIVE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 --workload c3 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/native_world1_c3.log 2>&1 || exit 1
