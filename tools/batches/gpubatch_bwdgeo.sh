# bn_bwd_partial: more blocks for the deep, narrow-M layers; parity + bench + serial kernel traces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/bg_tests.log 2>&1 || { tail -30 gpurun_out/bg_tests.log; exit 1; }
tail -n 1 gpurun_out/bg_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/bg_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bg_b.log').read().strip().splitlines()[-1]);print(d['value'], d['bf16_train']['value'])"
done
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bg_prof_fp32s -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/bg_prof_fp32s.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bg_prof_bf16s -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/bg_prof_bf16s.log 2>&1 || exit 1
echo done
