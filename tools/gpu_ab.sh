#!/bin/bash
# Same-box A/B of bench lines: AB="name:K=V&K=V;name2:..." WLS="c2 c3", then
# optional tests (TESTS="tests/x.py ..." TESTK=expr).  Output: gpurun_out/ab/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/ab"; mkdir -p "$O"
export TMPDIR=/tmp
# variants set LHPC_* knobs: only the tuning build reads them (make -C libhpc_amd/csrc tuning)
[ -f "$R/libhpc_amd/_lib_tuning/liblhpc.so" ] && export LHPC_LIB_PATH=${LHPC_LIB_PATH:-$R/libhpc_amd/_lib_tuning/liblhpc.so}
log() { echo "== $* $(date +%T)" >> "$O/progress.log"; }
IFS=';' read -ra VS <<< "${AB:-base:X=0}"
for rep in $(seq 1 ${REPS:-1}); do
  for WL in ${WLS:-c2}; do
    for V in "${VS[@]}"; do
      name=${V%%:*}; kv=${V#*:}
      log "bench $WL $name rep $rep"
      env $(echo "$kv" | tr '&' ' ') timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_${WL}_${name}_$rep.log" 2>&1 || { log "FAIL bench $WL $name"; exit 1; }
    done
  done
done
if [ -n "${TESTS:-}" ]; then
  log tests
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTK:+-k "$TESTK"} > "$O/pytest.log" 2>&1 || { log "FAIL tests"; exit 1; }
fi
log done
exit 0
