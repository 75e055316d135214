set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_spmv.py tests/test_gpu_stencil.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python tools/explore.py --only spmv > gpurun_out/explore2.log 2>&1
fi
exit $rc
