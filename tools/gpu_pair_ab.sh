#!/bin/bash
# Same-box A/B of the XTILE reduce pair mode (LHPC_XTILE_PAIR=0/1): SpMV GPU
# parity tests under both, then bench lines for $WLS, REPS times, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/pair"; mkdir -p "$O"
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
for P in 1 0; do
  LHPC_XTILE_PAIR=$P step pytest_p$P 600 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
done
for REP in ${REPS:-1 2}; do
  for P in 0 1; do
    for WL in ${WLS:-c2 c3 c4}; do
      LHPC_XTILE_PAIR=$P step bench_p${P}_${WL}_$REP 300 python bench.py --workload $WL --no-cpu-baseline || exit 1
    done
  done
done
exit 0
