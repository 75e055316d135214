#!/bin/bash
# round 4: consumer-side P2P waits + uploaded device builds — full GPU suite,
# the P2P rehearsals, the default bench (plan build times)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest.txt 2>&1 || exit 1
for n in 200000 2500000; do
  LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --n-rows $n --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/p2p_n$n.log 2>&1 || exit 1
done
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1 || exit 1
