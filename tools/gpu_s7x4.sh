#!/bin/bash
# stencil7 x4-ring A/B on C5: buf4 parity tests, then per-kernel times under env variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stencil.py -k "buf4 or c5_size or (every_impl and buf and staged)" > gpurun_out/s7x4_tests.log 2>&1 || { tail -30 gpurun_out/s7x4_tests.log; exit 1; }
tail -3 gpurun_out/s7x4_tests.log
WL=c5 VARIANTS=${VARIANTS:-"base:X=1;x4nt:LHPC_STENCIL7_IMPL=buf4"} bash tools/gpu_split.sh || exit 1
python tools/summ_split.py
