#!/bin/bash
# Per-kernel split of a bench workload under env variants (rocprofv3 kernel
# trace, one short run each): VARIANTS="name:K=V+K=V;name2:...".
# Output: gpurun_out/split/<name>/run_kernel_stats.csv + bench line logs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O="$R/gpurun_out/split"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
WL=${WL:-c2}
IFS=';' read -ra VS <<< "$VARIANTS"
for V in "${VS[@]}"; do
  name=${V%%:*}; kv=${V#*:}
  echo "== $name ($kv) $(date +%T)" >> "$O/progress.log"
  env $(echo "$kv" | tr '+' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run -f csv -- python3 "$R/bench.py" --workload $WL --steps 10 --warmup 3 --no-cpu-baseline > "$O/$name.log" 2>&1 || exit 1
done
exit 0
