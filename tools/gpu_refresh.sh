#!/bin/bash
# Refresh every bench workload's line + rocprofv3 kernel stats (one run each),
# and PMC FETCH/WRITE passes for $PMC_WLS.  Output under gpurun_out/refresh/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/refresh
export TMPDIR=/tmp
O="$R/gpurun_out/refresh"
cd /tmp
for WL in ${WLS:-c2 c3 c4 c5 blur_x blur_y sort cg}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL > "$O/bench_$WL.log" 2>&1 || exit 1
  echo "done $WL" >> "$O/progress.log"
done
for WL in ${PMC_WLS:-blur_x}; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch_$WL.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_write_$WL.log" 2>&1 || exit 1
  echo "pmc $WL" >> "$O/progress.log"
done
