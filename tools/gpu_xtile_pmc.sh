#!/bin/bash
# PMC passes on a bench workload (one counter group per run; groups separated
# by ';' in $PASSES).  Output under gpurun_out/xpmc/<workload>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O="$R/gpurun_out/xpmc"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
WL=${WL:-c2}
PASSES=${PASSES:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum"}
i=0
IFS=';' read -ra PGROUPS <<< "$PASSES"
for CTR in "${PGROUPS[@]}"; do
  i=$((i+1))
  echo "== $WL pass $i $CTR $(date +%T)" >> "$O/progress.log"
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$O/$WL/p$i" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 3 --warmup 1 --no-cpu-baseline > "$O/$WL.p$i.log" 2>&1 || exit 1
done
exit 0
