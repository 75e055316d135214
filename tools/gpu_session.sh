#!/bin/bash
# One box, in order (each GPU step under its own time limit, chained):
# sort tests on the product build, the full -m gpu suite + smoke, the default
# bench line, then same-box A/B bench lines ($AB over $WLS, tools/gpu_ab.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/session"; mkdir -p "$O"
export TMPDIR=/tmp
log() { echo "== $* $(date +%T)" >> "$O/progress.log"; }
if [ -z "${SKIP_SORT:-}" ]; then
  log sort-tests
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_sort.log" 2>&1 || { log FAIL sort-tests; exit 1; }
fi
if [ -z "${SKIP_SUITE:-}" ]; then
  log suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 || { log FAIL suite; exit 1; }
  log smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { log FAIL smoke; exit 1; }
  log bench
  timeout -k 10 300 python bench.py > "$O/bench_default.log" 2>&1 || { log FAIL bench; exit 1; }
fi
if [ -n "${AB:-}" ]; then
  log ab
  bash tools/gpu_ab.sh || { log FAIL ab; exit 1; }
fi
log done
exit 0
