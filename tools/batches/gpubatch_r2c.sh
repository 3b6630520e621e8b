# round 2: full GPU suite, smoke, default bench (drop-in predictor leg, fp32 inference leg, CPU legs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1 || { tail -40 gpurun_out/r2c_tests.log; exit 1; }
tail -n 2 gpurun_out/r2c_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1 || { tail -20 gpurun_out/r2c_smoke.log; exit 1; }
tail -n 1 gpurun_out/r2c_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r2c_bench.log 2>&1 || { tail -20 gpurun_out/r2c_bench.log; exit 1; }
tail -n 1 gpurun_out/r2c_bench.log
