#!/bin/bash
# round 4: bench's native N>1 path rehearsed with 2 ranks on one GPU (P2P windows,
# plain + chained steps), then the per-rank model with one / two reduce streams
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4g; mkdir -p $O
LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/rehearsal_p2p_c2.log 2>&1 || exit 1
timeout -k 10 400 python tools/explore_rank_model.py > $O/rank_model.jsonl 2> $O/rank_model.err || exit 1
