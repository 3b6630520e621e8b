# fp32 stems on the packed NHWC-4 layout: kernel + model parity, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/f_tests.log 2>&1 || { tail -30 gpurun_out/f_tests.log; exit 1; }
tail -n 1 gpurun_out/f_tests.log
MAUV_F32_STEM_PACK=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 > gpurun_out/f_bench0.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 > gpurun_out/f_bench1.log 2>&1 || exit 1
tail -n 1 gpurun_out/f_bench0.log | cut -c1-200; tail -n 1 gpurun_out/f_bench1.log | cut -c1-200
echo done
