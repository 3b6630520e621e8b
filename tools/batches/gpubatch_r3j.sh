# round 3: the full GPU suite and smoke() on the current state
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3j_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r3j_suite.log
grep -E "FAIL|Error" gpurun_out/r3j_suite.log | head -10
[ $rc -eq 0 ] || { echo "suite rc=$rc: stop"; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j_smoke.log 2>&1 || { tail -5 gpurun_out/r3j_smoke.log; exit 1; }
tail -2 gpurun_out/r3j_smoke.log
echo done
