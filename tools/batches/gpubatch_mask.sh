# 1-bit ReLU masks for block-output BNs (MAUV_BN_RELU_MASK): parity + A/B bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/mk_tests.log 2>&1 || { tail -30 gpurun_out/mk_tests.log; exit 1; }
tail -n 1 gpurun_out/mk_tests.log
for v in 0 1 0 1; do
MAUV_BN_RELU_MASK=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/mk_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/mk_b.log').read().strip().splitlines()[-1]);print('mask=$v', d['value'], d['bf16_train']['value'])"
done
echo done
