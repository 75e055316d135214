#!/bin/bash
# XTILE vs XSLICE on uniform 15/row matrices as n grows (x tiles S = n/W):
# gpurun_out/r4c/{xtile,xslice}_<dtype>_<n>.log; NS = the sizes, DT = f32/f64
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r4c
DT=${DT:-f32}
for n in ${NS:-20000000 40000000 80000000 150000000}; do
  timeout -k 10 300 python bench.py --n $n --dtype $DT --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r4c/xtile_${DT}_$n.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --n $n --dtype $DT --no-cpu-baseline --steps 10 --warmup 2 --spmv-options '{"spmv_no_xtile": 1}' > gpurun_out/r4c/xslice_${DT}_$n.log 2>&1 || exit 1
done
