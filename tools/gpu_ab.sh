#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_spmv.log 2>&1 || exit 1
timeout -k 10 600 python tools/explore.py --only spmv > gpurun_out/explore3.log 2>&1
