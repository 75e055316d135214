#!/bin/bash
# round 4: column blocks re-swept after the register-row-offset reduce (fp32
# G = 2 keeps 4 blocks per CU up to ≈ 975 tiles): n = 80M B = 2 / 3 / 4 and
# n = 150M B = 3 / 4 / 5, same box, two runs each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4cb; mkdir -p $O
B="timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 2"
for i in 1 2; do
  for cfg in "80000000 2 3 4" "150000000 3 4 5"; do
    set -- $cfg
    n=$1; shift
    for b in "$@"; do
      $B --n-rows $n --spmv-options "{\"xtile_col_blocks\": $b}" >> $O/f32_${n}_b$b.log 2>&1 || exit 1
    done
  done
done
