#!/bin/bash
# round 4: device-input plans of row parts / column blocks — GPU tests, then
# the n = 80M / 150M bench lines (device-built plan timed beside the host one,
# layouts compared by digest).  gpurun_out/r4l/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spmv.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "device_input or col_blocks or coo_to_csr" > $O/pytest.txt 2>&1 || exit 1
for n in 80000000 150000000; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --n $n > $O/bench_$n.log 2>&1 || exit 1
done
