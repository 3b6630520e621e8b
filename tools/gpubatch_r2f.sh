set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_staging_metrics_gpu.py tests/test_standalone_gpu.py tests/test_integration_gpu.py tests/test_dropin_gpu.py tests/test_kernels_gpu.py -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r2f_tests.log
exit $rc
