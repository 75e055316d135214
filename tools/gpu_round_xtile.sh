#!/bin/bash
# One box: XTILE scaling explore (rank-0 chunk plans at W = 1..8), the 2-rank
# gloo rehearsal of bench.py --gpus 2 (c2), refreshed bench lines + kernel
# stats for c2/c3/c4 (with CPU baselines), and FETCH/WRITE PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/rx"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
[ "${SKIP_SCALING:-0}" = 1 ] || step scaling 300 python tools/explore_scaling.py || exit 1
[ "${SKIP_DIST:-0}" = 1 ] || LHPC_DIST_BACKEND=gloo step rehearsal_c2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload c2 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
cd /tmp
for WL in ${WLS:-c2 c3 c4}; do
  step bench_$WL 600 rocprofv3 --kernel-trace --stats -d "$O/stats_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL || exit 1
done
for WL in ${PMC_WLS:-c2 c3 c4}; do
  step pmcf_$WL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline || exit 1
  step pmcw_$WL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline || exit 1
done
exit 0
