# round 3: new parity / configs[4] / KL / multi-rank bench tests (calibration prints), the full
# GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kl_gpu.py tests/test_parity16_gpu.py tests/test_configs4_gpu.py tests/test_bench_ranks_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r3a_new.log 2>&1
rc=$?
tail -n 40 gpurun_out/r3a_new.log
case $rc in 0|1) ;; *) echo "new tests rc=$rc: stop"; exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_parity16_gpu.py --deselect tests/test_configs4_gpu.py --deselect tests/test_bench_ranks_gpu.py --deselect tests/test_kl_gpu.py > gpurun_out/r3a_suite.log 2>&1
rc=$?
tail -n 5 gpurun_out/r3a_suite.log
case $rc in 0|1) ;; *) echo "suite rc=$rc: stop"; exit $rc;; esac
timeout -k 10 600 python -u bench.py > gpurun_out/r3a_bench.log 2>&1 || exit 1
tail -c 3000 gpurun_out/r3a_bench.log
echo done
