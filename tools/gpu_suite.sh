#!/bin/bash
# Full GPU suite + smoke (what the driver runs at round end).  gpurun_out/suite/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/suite"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)" >> "$O/progress.log";
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
  echo "== $name rc=$rc $(date +%T)" >> "$O/progress.log"; return $rc; }
step pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTK:+-k "$TESTK"} || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
exit 0
