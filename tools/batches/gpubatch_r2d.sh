set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r2d_tests.log
exit $rc
