#!/bin/bash
# GPU sort / COO→CSR tests (+ optional bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_sort.py -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_sort.log 2>&1 || exit 1
if [ -n "${SORT_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py --workload sort ${SORT_BENCH} > gpurun_out/bench_sort.log 2>&1 || exit 1
fi
