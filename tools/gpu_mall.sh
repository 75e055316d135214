#!/bin/bash
# Infinity-Cache round-trip probe + C2 baseline bench on this box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O="$R/gpurun_out/mall"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 240 ./tools/_build/mall_probe > "$O/mall_probe.jsonl" 2> "$O/mall_probe.err" || exit 1
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > "$O/bench_c2.log" 2>&1 || exit 1
exit 0
