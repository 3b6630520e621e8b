# round 2 start: GPU tests + default bench on the restored tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1 || { tail -30 gpurun_out/r2a_tests.log; exit 1; }
tail -n 1 gpurun_out/r2a_tests.log
timeout -k 10 900 python -u bench.py --infer-fp32 > gpurun_out/r2a_bench.log 2>&1 || { tail -20 gpurun_out/r2a_bench.log; exit 1; }
tail -n 1 gpurun_out/r2a_bench.log
