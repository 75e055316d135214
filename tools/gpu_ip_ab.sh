#!/bin/bash
# iperm reduce A/B: SpMV GPU tests (all layouts), then C2/C3 call times for
# the perm reduce (LHPC_XTILE_IPERM=0), the default iperm reduce, and the
# library variants under libhpc_amd/_ab/<name>/ ($VARS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/ip"; mkdir -p "$O"
L=libhpc_amd/_lib/liblhpc.so; cp "$L" "$O/cur.so.bak"
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 || exit 1
for REP in ${REPS:-1 2}; do
  for V in perm ip ${VARS}; do
    if [ -d "libhpc_amd/_ab/$V" ]; then cp "libhpc_amd/_ab/$V/liblhpc.so" "$L"; else cp "$O/cur.so.bak" "$L"; fi
    IP=1; [ "$V" = perm ] && IP=0
    for WL in ${WLS:-c2 c3}; do
      LHPC_XTILE_IPERM=$IP timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > "$O/b_${V}_${WL}_$REP.log" 2>&1 || { cp "$O/cur.so.bak" "$L"; exit 1; }
      echo "$V $WL $REP $(grep -o '"call_us": [0-9.]*' "$O/b_${V}_${WL}_$REP.log")" >> "$O/summary.txt"
    done
  done
done
cp "$O/cur.so.bak" "$L"
exit 0
