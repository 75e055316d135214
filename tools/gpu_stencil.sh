#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_stencil.py tests/test_layout.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_stencil.log 2>&1 || exit 1
timeout -k 10 600 python tools/explore_stencil.py > gpurun_out/explore_stencil.log 2>&1
