#!/bin/bash
# round 4: fp64 XTILE reduce pulling a later chunk's segment-table row,
# base row and descriptor into L2 (LHPC_XT_PF64 = chunks ahead: 0 = off, 32,
# 64 = the build's default, 128) — fp64 XTILE tests on the default build,
# then same-box C3 / fp64 C4 bench lines, two runs each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4pf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmv.py -x -q -p no:cacheprovider -k "f64 or c3" \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --dtype f64"
for i in 1 2; do
  for wl in c3 c4; do
    for v in 0 32 128; do
      LHPC_LIB_PATH=$R/libhpc_amd/_lib_pf$v/liblhpc.so $B --workload $wl >> $O/pf${v}_$wl.log 2>&1 || exit 1
    done
    $B --workload $wl >> $O/pf64_$wl.log 2>&1 || exit 1
  done
done
