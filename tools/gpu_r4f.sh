#!/bin/bash
# round-4 checks: device-input layout, row parts past int32, XSLICE large grid, C++ API, multi/dist
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spmv.py tests/test_layout.py tests/test_gpu_multi.py tests/test_gpu_dist.py -k "device_input or coo_to_csr_to_spmv or parts or xslice_dispatch or cpp_api or multi or cg or chain" -x -q -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 20000000 --per-row 108 --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_parts.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 80000000 --no-cpu-baseline --steps 10 --warmup 2 --spmv-options '{"spmv_no_xtile": 1}' > $O/xslice_80m.log 2>&1
