#!/bin/bash
# round 4: ADAPTIVE row blocks of up to 512 rows (two rows per lane past
# 256) against the 256-row blocks (_lib_a256: -DLHPC_ADAPT_ROWS=256) — CG /
# ADAPTIVE GPU tests on the new build, then same-box A/B of the CG bench
# (4096² Laplacian, fp64), three runs each, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4z; mkdir -p $O
V=$R/libhpc_amd/_lib_a256/liblhpc.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_cg.py tests/test_gpu_spmv.py -x -q -p no:cacheprovider \
  -k "cg or adaptive or dot or c1 or small" --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
for wl in cg; do
  for i in 1 2 3; do
    $B --workload $wl --steps 40 --warmup 5 >> $O/new_$wl.log 2>&1 || exit 1
    LHPC_LIB_PATH=$V $B --workload $wl --steps 40 --warmup 5 >> $O/a256_$wl.log 2>&1 || exit 1
  done
done
