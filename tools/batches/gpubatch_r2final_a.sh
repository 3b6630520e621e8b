# round-2 evidence, part A: the full GPU suite and smoke()
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2final_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r2final_tests.log | head; tail -5 gpurun_out/r2final_tests.log; exit 1; }
tail -1 gpurun_out/r2final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2final_smoke.log 2>&1 || { tail -20 gpurun_out/r2final_smoke.log; exit 1; }
tail -1 gpurun_out/r2final_smoke.log
