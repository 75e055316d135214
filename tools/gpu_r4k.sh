#!/bin/bash
# round 4: XTILE column blocks — how many: forced B per size (same box).
# gpurun_out/r4k/<dtype>_<n>_b<B>.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4k; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2"
for cfg in ${CFGS:-"f32 10000000 1 2" "f32 40000000 2 3 4" "f32 80000000 2 3 4 6" "f32 150000000 2 3 4" "f64 10000000 1 2" "f64 40000000 3 4 6"}; do
  set -- $cfg
  dt=$1; n=$2; shift 2
  for b in "$@"; do
    $B --dtype $dt --n $n --spmv-options "{\"xtile_col_blocks\": $b}" > $O/${dt}_${n}_b$b.log 2>&1 || exit 1
  done
done
