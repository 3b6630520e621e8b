# session-3 re-entry check: full GPU suite, smoke(), default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/s3a_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/s3a_tests.log | head; tail -5 gpurun_out/s3a_tests.log; exit 1; }
tail -1 gpurun_out/s3a_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3a_smoke.log 2>&1 || { tail -20 gpurun_out/s3a_smoke.log; exit 1; }
tail -1 gpurun_out/s3a_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s3a_bench.log 2>&1 || { tail -20 gpurun_out/s3a_bench.log; exit 1; }
tail -1 gpurun_out/s3a_bench.log
