#!/bin/bash
# round 4: chunk row offsets in registers for the fp32 G = 2 reduce (and the
# G = 1 plans whose LDS row offsets cost a block per CU) — XTILE GPU tests,
# then same-box A/B against the previous build (_lib_prev) at C2, n = 20M /
# 30M and 80M
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_dist.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3"
for n in 10000000 20000000 30000000 80000000; do
  for i in 1 2; do
    $B --n $n >> $O/new_$n.log 2>&1 || exit 1
    LHPC_LIB_PATH=$R/libhpc_amd/_lib_prev/liblhpc.so $B --n $n >> $O/prev_$n.log 2>&1 || exit 1
  done
done
