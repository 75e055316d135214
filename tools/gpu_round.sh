#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (JSON line), rocprofv3 stats.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name" >> "$R/gpurun_out/round.log"
  timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> "$R/gpurun_out/round.log"
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 1000 python -m pytest tests -m gpu -x -q -p no:cacheprovider || exit 1
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py || exit 1
  cd /tmp
  step prof_bench 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  cd "$R"
fi
exit 0
