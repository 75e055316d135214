#!/bin/bash
# Profiling session: A/B explore, kernel-trace stats of bench, PMC traffic passes.
# PMC passes run with counters only (no sys/runtime trace), one counter group each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
WL=${1:-c2}
run() { local name=$1 secs=$2; shift 2; echo "== $name" >> "$R/gpurun_out/prof_round.log";
  timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc" >> "$R/gpurun_out/prof_round.log"; return $rc; }
if [ "${SKIP_EXPLORE:-0}" != 1 ]; then
  run explore_ab 600 python tools/explore.py --only spmv || exit 1
fi
cd /tmp
run prof_stats_$WL 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_stats_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run pmc_fetch_$WL 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline || exit 1
if [ "${CALIB:-0}" = 1 ]; then
  run pmc_calib 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_calib" -o run -f csv -- python3 "$R/tools/pmc_calibrate.py" || exit 1
fi
run pmc_write_$WL 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write_$WL" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline || exit 1
exit 0
