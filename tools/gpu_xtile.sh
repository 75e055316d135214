#!/bin/bash
# XTILE bring-up: parity tests, then C2/C3/C4 bench lines (XTILE vs XSLICE) and
# a kernel-trace profile of the C2 bench.  Output under gpurun_out/xtile/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/xtile"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest 600 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "${TESTK:-xtile}" || exit 1
[ "${TESTS_ONLY:-0}" = 1 ] && exit 0
for WL in ${WLS:-c2 c3 c4}; do
  step bench_$WL 600 python bench.py --workload $WL --no-cpu-baseline || exit 1
done
# A/B variants: "name:K=V,K=V;..." (default: the tile-stream XTILE layout)
IFS=';' read -ra VS <<< "${AB_VARIANTS-seg:LHPC_XTILE_LAYOUT=seg}"
for V in "${VS[@]}"; do
  name=${V%%:*}; kv=${V#*:}
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > "$O/bench_c2_$name.log" 2>&1 || exit 1
done
cd /tmp
step prof_c2 600 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o run -f csv -- python3 "$R/bench.py" --workload c2 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
exit 0
