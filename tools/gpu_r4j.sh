#!/bin/bash
# round 4: XTILE column blocks — GPU tests, then same-box A/B of auto
# (column blocks) against one block as n grows.  gpurun_out/r4j/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spmv.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "col_blocks or row_parts or large_n or parts_past or golden" > $O/pytest.txt 2>&1 || exit 1
[ "${TESTS_ONLY:-0}" = 1 ] && exit 0
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2"
for cfg in "f32 40000000" "f32 56000000" "f32 80000000" "f64 20000000" "f64 40000000" "f32 150000000"; do
  set -- $cfg
  $B --dtype $1 --n $2 > $O/auto_$1_$2.log 2>&1 || exit 1
  $B --dtype $1 --n $2 --spmv-options '{"xtile_col_blocks": 1}' > $O/one_$1_$2.log 2>&1 || exit 1
done
