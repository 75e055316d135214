#!/bin/bash
# Direct peer exchange (lhpc_dist_p2p_*) on one GPU: the two-process test,
# then bench.py --gpus 2 as two ranks sharing cuda:0 over gloo with
# LHPC_DIST_P2P=1 (IPC windows, RCCL-free local communicators).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/p2p"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
step pytest 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 step bench_p2p 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --workload c2 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
exit 0
