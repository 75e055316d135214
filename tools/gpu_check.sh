#!/bin/bash
# Round-3 GPU check: the -m gpu suite + smoke, then bench.py's N>1 paths
# rehearsed on the 1-GPU box: 2 gloo ranks sharing cuda:0 with the peer
# exchange (LHPC_DIST_P2P=1), and the native RCCL path at world 1
# (LHPC_DIST_NATIVE=1).  Output: gpurun_out/check/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/check"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
if [ -z "${SKIP_SUITE:-}" ]; then
  step pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTK:+-k "$TESTK"} || exit 1
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
step rehearsal_p2p 600 env LHPC_DIST_BACKEND=gloo LHPC_DIST_P2P=1 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload c2 --steps 10 \
  --warmup 2 --no-cpu-baseline || exit 1
step native_world1 600 env LHPC_DIST_NATIVE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --workload c3 --steps 10 --warmup 2 \
  --no-cpu-baseline || exit 1
exit 0
