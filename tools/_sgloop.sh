mkdir -p gpurun_out/sgloop
for i in $(seq 1 25); do
  timeout -k 5 60 tests/cpp/_build/test_sparse_grid gpu > gpurun_out/sgloop/run_$i.log 2>&1
  echo "$i rc=$?" >> gpurun_out/sgloop/summary.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sgloop/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sgloop/smoke.log 2>&1
