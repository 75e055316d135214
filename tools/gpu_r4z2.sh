#!/bin/bash
# round 4: ADAPTIVE rows per block 64 / 128 / 256 / 512 on the CG bench
# (4096² Laplacian fp64), same box, three runs each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4z2; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --workload cg --steps 40 --warmup 5"
for i in 1 2 3; do
  for v in 64 128 256; do
    LHPC_LIB_PATH=$R/libhpc_amd/_lib_a$v/liblhpc.so $B >> $O/a$v.log 2>&1 || exit 1
  done
  $B >> $O/a512.log 2>&1 || exit 1
done
