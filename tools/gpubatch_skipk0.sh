# dgrad: skip tapless accumulate-only parity classes; parity + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/k0_tests.log 2>&1 || { tail -30 gpurun_out/k0_tests.log; exit 1; }
tail -n 1 gpurun_out/k0_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/k0_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/k0_b.log').read().strip().splitlines()[-1]);print(d['value'], d['bf16_train']['value'])"
done
echo done
