#!/bin/bash
# stencil GPU tests, then the C5 profile refresh: kernel-trace stats bench line,
# FETCH_SIZE / WRITE_SIZE passes and the FETCH_SIZE calibration pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stencil.py tests/test_dist_stencil.py -m gpu > gpurun_out/s7_tests.log 2>&1 || { tail -30 gpurun_out/s7_tests.log; exit 1; }
tail -2 gpurun_out/s7_tests.log
WLS=c5 bash tools/gpu_prof_stencil.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_calib" -o run -f csv -- python3 "$R/tools/pmc_calibrate.py" > "$R/gpurun_out/pmc_calib.log" 2>&1 || exit 1
grep '^{' "$R/gpurun_out/prof_stats_c5.log"
