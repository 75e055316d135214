#!/bin/bash
# Same-box A/B of library variants: for each libhpc_amd/_ab/<name>.so (plus the
# tree's own build as "cur"), the SpMV GPU parity tests, then bench lines for
# $WLS.  Output under gpurun_out/ab/.  Variants: VARS="cur old b1024" (a
# directory name means _ab/<name>/liblhpc.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/ab"; mkdir -p "$O"
L=libhpc_amd/_lib/liblhpc.so; cp "$L" "$O/cur.so.bak"
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
for REP in ${REPS:-1}; do
for V in ${VARS:-cur}; do
  if [ "$V" = cur ]; then cp "$O/cur.so.bak" "$L"; elif [ -d "libhpc_amd/_ab/$V" ]; then cp "libhpc_amd/_ab/$V/liblhpc.so" "$L"; else cp "libhpc_amd/_ab/$V.so" "$L"; fi
  if [ "$REP" = 1 ] && [ "${TESTS:-1}" = 1 ] && [ "$V" != old ]; then
    step pytest_$V 600 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
  fi
  for WL in ${WLS:-c3 c2}; do
    step bench_${V}_${WL}_$REP 300 python bench.py --workload $WL --no-cpu-baseline || exit 1
  done
done
done
cp "$O/cur.so.bak" "$L"
exit 0
