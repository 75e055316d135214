#!/bin/bash
# Kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes for the stencil workloads (one counter per pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
for WL in ${WLS:-c5 blur_x blur_y}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_stats_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 20 --warmup 5 > "$R/gpurun_out/prof_stats_$WL.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_fetch_$WL.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_write_$WL.log" 2>&1 || exit 1
  echo "done $WL"
done
