#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_stencil.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_stencil.log 2>&1 || exit 1
timeout -k 10 600 python tools/explore_stencil.py > gpurun_out/explore_stencil.log 2>&1 || exit 1
cd /tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_stencil" -o run -f csv -- python3 "$R/tools/explore_stencil.py" > "$R/gpurun_out/pmc_stencil.log" 2>&1 || exit 1
