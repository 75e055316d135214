#!/bin/bash
# round 4: CG graph blocks — CG GPU tests, the A/B of issue paths, bench cg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cg.py tests/test_debug_build.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python tools/explore_cg_graph.py > $O/ab.jsonl 2> $O/ab.err || exit 1
timeout -k 10 300 python bench.py --workload cg --no-cpu-baseline > $O/bench_cg.log 2>&1 || exit 1
