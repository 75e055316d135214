#!/bin/bash
# round 4: column blocks below the 768-tile threshold (LDS: above ≈ 475 tiles
# the fp32 reduce fits 3 blocks per CU instead of 4) — forced B = 1 / 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4w; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2"
for cfg in ${CFGS:-"f32 20000000" "f32 30000000" "f64 15000000"}; do
  set -- $cfg
  for b in ${BS:-1 2 1 2}; do
    $B --dtype $1 --n $2 --spmv-options "{\"xtile_col_blocks\": $b}" >> $O/${1}_${2}_b$b.log 2>&1 || exit 1
  done
done
