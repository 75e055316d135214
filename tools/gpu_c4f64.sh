#!/bin/bash
# C4 in fp64: bench line under rocprofv3 --kernel-trace --stats,
# then FETCH/WRITE PMC passes and the 4-B fetch calibration.  Output under
# gpurun_out/c4f64/; tools/pmc_traffic.py c4f64_xtile ... turns the passes into
# profiles/traffic.json's entry.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O="$R/gpurun_out/c4f64"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run -f csv -- python3 "$R/bench.py" --workload c4 --dtype f64 > "$O/bench.log" 2>&1 || exit 1
echo stats >> "$O/progress.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_calib" -o run -f csv -- python3 "$R/tools/pmc_calibrate.py" > "$O/calib.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -f csv -- python3 "$R/bench.py" --workload c4 --dtype f64 --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -f csv -- python3 "$R/bench.py" --workload c4 --dtype f64 --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_write.log" 2>&1 || exit 1
echo done >> "$O/progress.log"
