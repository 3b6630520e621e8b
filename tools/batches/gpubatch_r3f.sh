# round 3: BN-backward fold prototype — tolerance test and interleaved A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels16_gpu.py -k fold -v -s --timeout 200 --timeout-method thread > gpurun_out/r3f_test.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r3f_test.log | tail -20
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
timeout -k 10 400 python -u tools/fold_ab.py --dtype bf16 > gpurun_out/r3f_fold_ab_bf16.log 2>&1 || { tail -20 gpurun_out/r3f_fold_ab_bf16.log; exit 1; }
cat gpurun_out/r3f_fold_ab_bf16.log
echo done
