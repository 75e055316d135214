#!/bin/bash
# round 4 same-box A/Bs: (1) sort scratch from the library pool vs the device's
# default pool (_lib_rbdp); (2) fp32 XTILE reduce with 1024-thread blocks /
# 16384-nonzero chunks (_lib_rb1024) against 512 / 8192 as n grows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4h; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
for i in 1 2; do
  $B --workload sort --steps 20 > $O/sort_pool_$i.log 2>&1 || exit 1
  LHPC_LIB_PATH=$R/libhpc_amd/_lib_rbdp/liblhpc.so $B --workload sort --steps 20 > $O/sort_dflt_$i.log 2>&1 || exit 1
done
for n in 10000000 40000000 80000000; do
  for i in 1 2; do
    $B --n $n --steps 10 --warmup 2 > $O/m512_${n}_$i.log 2>&1 || exit 1
    LHPC_LIB_PATH=$R/libhpc_amd/_lib_rb1024/liblhpc.so $B --n $n --steps 10 --warmup 2 > $O/m1024_${n}_$i.log 2>&1 || exit 1
  done
done
# FETCH_SIZE calibration for tools/pmc_traffic.py (the 4-B/lane read factor)
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_calib" -o run -f csv -- python3 "$R/tools/pmc_calibrate.py" > "$R/$O/pmc_calib.log" 2>&1 || exit 1
