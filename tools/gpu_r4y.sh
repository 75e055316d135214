#!/bin/bash
# round 4: fp64 XTILE reduce with 512-thread blocks over 4096-nonzero chunks
# (LHPC_XT_RBLK64=512: 4 blocks per CU) against the kept 1024-thread form —
# fp64 XTILE tests on the variant, then same-box A/B of C3 (fp64) and fp64
# power-law C4, three runs each, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4y; mkdir -p $O
V=$R/libhpc_amd/_lib_r64/liblhpc.so
LHPC_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_spmv.py -x -q -p no:cacheprovider -k "f64 or c3" \
  --timeout 300 --timeout-method thread > $O/pytest_r64.txt 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3"
for wl in c3 c4; do
  for i in 1 2 3; do
    $B --workload $wl --dtype f64 >> $O/kept_$wl.log 2>&1 || exit 1
    LHPC_LIB_PATH=$V $B --workload $wl --dtype f64 >> $O/r64_$wl.log 2>&1 || exit 1
  done
done
