#!/bin/bash
# A/B with per-kernel stats: AB="name:K=V&...;..." WLS="c2": each variant's bench
# line under rocprofv3 --kernel-trace --stats.  Output: gpurun_out/abp/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O="$R/gpurun_out/abp"; mkdir -p "$O"
export TMPDIR=/tmp
# variants set LHPC_* knobs: only the tuning build reads them (make -C libhpc_amd/csrc tuning)
[ -f "$R/libhpc_amd/_lib_tuning/liblhpc.so" ] && export LHPC_LIB_PATH=${LHPC_LIB_PATH:-$R/libhpc_amd/_lib_tuning/liblhpc.so}
cd /tmp
IFS=';' read -ra VS <<< "${AB:-base:X=0}"
for rep in $(seq 1 ${REPS:-1}); do
  for WL in ${WLS:-c2}; do
    for V in "${VS[@]}"; do
      name=${V%%:*}; kv=${V#*:}
      for e in $(echo "$kv" | tr '&' ' '); do export "$e"; done
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${WL}_${name}_$rep" -o run -f csv -- python3 "$R/bench.py" --workload $WL --no-cpu-baseline --steps ${STEPS:-50} > "$O/bench_${WL}_${name}_$rep.log" 2>&1 || { echo "FAIL $WL $name" >> "$O/progress.log"; exit 1; }
      for e in $(echo "$kv" | tr '&' ' '); do unset "${e%%=*}"; done
      echo "done $WL $name $rep" >> "$O/progress.log"
    done
  done
done
