# round 2: drop-in golden tests + the extended model parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_dropin_gpu.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1; rc=$?
tail -40 gpurun_out/r2b_tests.log
exit $rc
