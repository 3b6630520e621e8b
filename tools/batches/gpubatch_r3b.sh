# round 3: re-run the new tests after the fixes (calibration prints) and the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kl_gpu.py tests/test_resize.py tests/test_parity16_gpu.py tests/test_configs4_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r3b_new.log 2>&1
rc=$?
grep -E "PASS|FAIL|cos vs|dlogit|classes|KL |S=" gpurun_out/r3b_new.log | tail -40
case $rc in 0|1) ;; *) echo "new tests rc=$rc: stop"; exit $rc;; esac
timeout -k 10 700 python -u bench.py > gpurun_out/r3b_bench.log 2>&1 || { tail -20 gpurun_out/r3b_bench.log; exit 1; }
tail -c 2500 gpurun_out/r3b_bench.log
echo done
