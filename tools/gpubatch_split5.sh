# split kernel codegen fixes: parity + timing + bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_math_gpu.py tests/test_kernels_gpu.py > gpurun_out/s5_kern.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 30 > gpurun_out/s5_cb.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 30 --fused > gpurun_out/s5_cbf.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_model_gpu.py > gpurun_out/s5_model.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --steps 4 --warmup 1 > gpurun_out/s5_bench.log 2>&1 || exit 1
echo done
