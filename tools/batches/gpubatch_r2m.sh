# full GPU suite + smoke + one bench after the stem GEMM and the toggle cleanup
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2m_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r2m_tests.log | head -30; tail -30 gpurun_out/r2m_tests.log; exit 1; }
tail -1 gpurun_out/r2m_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2m_smoke.log 2>&1 || { tail -20 gpurun_out/r2m_smoke.log; exit 1; }
tail -2 gpurun_out/r2m_smoke.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r2m_bench.log 2>&1 || { tail -20 gpurun_out/r2m_bench.log; exit 1; }
tail -1 gpurun_out/r2m_bench.log | cut -c1-600
