# row-walk BN apply / backward-apply kernels: parity, A/B bench (MAUV_BN_ROWS=0 = grid-stride), kernel traces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/br_tests.log 2>&1 || { tail -30 gpurun_out/br_tests.log; exit 1; }
tail -n 1 gpurun_out/br_tests.log
for v in 0 1 0 1; do
MAUV_BN_ROWS=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/br_b$v.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/br_b$v.log').read().strip().splitlines()[-1]);print('rows=$v', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/br_prof_bf16s -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/br_prof_bf16s.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/br_prof_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/br_prof_inf.log 2>&1 || exit 1
echo done
