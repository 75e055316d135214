#!/bin/bash
# Full round: all GPU tests, smoke, default bench, per-workload benches + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "== $name" >> "$R/gpurun_out/full.log";
  timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc" >> "$R/gpurun_out/full.log"; return $rc; }
run pytest_gpu 1000 python -m pytest tests -m gpu -x -q -p no:cacheprovider || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 600 python bench.py || exit 1
cd /tmp
for wl in c2 c3 c4 c5 blur_x blur_y; do
  run stats_$wl 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/stats_$wl" -o run -f csv -- python3 "$R/bench.py" --workload $wl --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
exit 0
