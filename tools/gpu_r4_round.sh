#!/bin/bash
# round 4 evidence session: full GPU suite + smoke, the default bench line,
# every bench workload under rocprofv3 kernel stats, FETCH/WRITE passes for
# $PMC_WLS.  Each GPU step has its own limit; the first failure ends the run.
# Output under gpurun_out/r4r/.  STAGES="tests bench stats pmc" selects parts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/r4r"; mkdir -p "$O"
export TMPDIR=/tmp
STAGES=${STAGES:-"tests bench stats pmc"}
has() { [[ " $STAGES " == *" $1 "* ]]; }
log() { echo "$(date +%T) $*" >> "$O/progress.log"; }
if has tests; then
  log pytest
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.txt" 2>&1 || exit 1
  log smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
fi
if has bench; then
  log bench
  timeout -k 10 600 python bench.py > "$O/bench_default.log" 2>&1 || exit 1
fi
cd /tmp
if has stats; then
  for WL in ${WLS:-c2 c3 c4 c5 blur_x blur_y sort cg}; do
    log "stats $WL"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats_$WL" -o run -f csv -- \
      python3 "$R/bench.py" --workload $WL > "$O/bench_$WL.log" 2>&1 || exit 1
  done
fi
if has pmc; then
  for WL in ${PMC_WLS:-c2}; do
    log "pmc $WL"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$WL" -o run -f csv -- \
      python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch_$WL.log" 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$WL" -o run -f csv -- \
      python3 "$R/bench.py" --workload $WL --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_write_$WL.log" 2>&1 || exit 1
  done
fi
log done
exit 0
