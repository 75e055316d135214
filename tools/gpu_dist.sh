#!/bin/bash
# Native multi-GPU layer on a 1-GPU box: lhpc_dist_* GPU tests, then bench.py's
# N > 1 code paths as far as one GPU allows — the native RCCL path at world 1
# (LHPC_DIST_NATIVE=1 under torch.distributed.run) for c2/c3/c5, and the
# torch-collective path as 2 gloo ranks sharing the GPU.  gpurun_out/dist/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/dist"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
step tests 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
port=29531
for WL in ${WLS:-c2 c3 c5}; do
  port=$((port+1))
  LHPC_DIST_NATIVE=1 step native_$WL 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --workload $WL --steps 10 --warmup 2 --no-cpu-baseline || exit 1
done
LHPC_DIST_BACKEND=gloo step gloo2_c2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --workload c2 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
exit 0
