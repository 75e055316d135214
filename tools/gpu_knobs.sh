#!/bin/bash
# Runtime-knob sweep of one workload (env settings from $KNOBS, ';'-separated,
# each a space-separated list of VAR=VALUE; "-" = defaults).  gpurun_out/knobs/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/knobs"; mkdir -p "$O"
i=0
IFS=';' read -ra SETS <<< "${KNOBS:--}"
for REP in ${REPS:-1}; do
  for S in "${SETS[@]}"; do
    i=$((i + 1)); E=(); [ "$S" != "-" ] && read -ra E <<< "$S"
    echo "== $i [$S] $(date +%T)" >> "$O/progress.log"
    env "${E[@]}" timeout -k 10 300 python bench.py --workload ${WL:-c3} --no-cpu-baseline > "$O/run_$i.log" 2>&1 || exit 1
    echo "$i|$S|$(grep -o '"call_us": [0-9.]*' "$O/run_$i.log")" >> "$O/summary.txt"
  done
done
exit 0
