# split-fp32 conv arithmetic: parity (kernel + model), per-shape timing split vs exact, bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_math_gpu.py tests/test_kernels_gpu.py > gpurun_out/split_kern.log 2>&1 &&
timeout -k 10 300 env MAUV_F32_MATH=exact python -u tools/conv_bench.py --reps 3 --top 12 > gpurun_out/cb_exact.log 2>&1 &&
timeout -k 10 300 env MAUV_F32_MATH=split python -u tools/conv_bench.py --reps 3 --top 12 > gpurun_out/cb_split.log 2>&1 &&
timeout -k 10 300 env MAUV_F32_MATH=split3 python -u tools/conv_bench.py --reps 3 --top 12 > gpurun_out/cb_split3.log 2>&1 &&
timeout -k 10 600 $T tests/test_model_gpu.py > gpurun_out/split_model.log 2>&1 &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --steps 4 --warmup 1 > gpurun_out/split_bench.log 2>&1
echo "exit $?"
