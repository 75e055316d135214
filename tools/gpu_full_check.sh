#!/bin/bash
# Full GPU suite + smoke, then the XTILE refresh (bench lines under kernel
# trace, PMC traffic).  Output under gpurun_out/full/ and gpurun_out/rx/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/full"; mkdir -p "$O"
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
SKIP_SCALING=${SKIP_SCALING:-1} SKIP_DIST=${SKIP_DIST:-0} bash tools/gpu_round_xtile.sh || exit 1
