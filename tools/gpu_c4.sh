#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_spmv2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload blur_x > gpurun_out/bench_blur_x.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload blur_y > gpurun_out/bench_blur_y.log 2>&1 || exit 1
