#!/bin/bash
# One run of tools/race_diag.hip (the round-2 host-path race):
# hipcc -O2 tools/race_diag.hip -o tools/_build/race_diag beforehand.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/race
timeout -k 10 300 ./tools/_build/race_diag ${ITERS:-2000} > gpurun_out/race/race_diag.jsonl 2> gpurun_out/race/race_diag.err
