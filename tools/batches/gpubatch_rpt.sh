# BN rows-per-thread sweep: apply (MAUV_BN_APPLY_RPT) and backward partial (MAUV_BN_PARTIAL_RPT)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py -k "bn" > gpurun_out/rp_tests.log 2>&1 || { tail -30 gpurun_out/rp_tests.log; exit 1; }
tail -n 1 gpurun_out/rp_tests.log
for cfg in "8 16" "4 16" "16 16" "8 8" "4 8" "8 16"; do
set -- $cfg
MAUV_BN_APPLY_RPT=$1 MAUV_BN_PARTIAL_RPT=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/rp_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/rp_b.log').read().strip().splitlines()[-1]);print('apply=$1 partial=$2', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
echo done
