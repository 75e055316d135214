#!/bin/bash
# round 4: fused P2P kernels (push + DONE signal, DONE wait + acquire) —
# the dist GPU tests, then the P2P rehearsal overhead runs of gpu_r4m.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_multi.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
for n in 200000 2500000; do
  LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --n-rows $n --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/p2p_n$n.log 2>&1 || exit 1
done
LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/p2p_c2.log 2>&1 || exit 1
