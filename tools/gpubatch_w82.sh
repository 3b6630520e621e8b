set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
MAUV_SPLIT_W8=2 timeout -k 10 400 $T tests/test_f32_math_gpu.py tests/test_kernels_gpu.py > gpurun_out/w82_kern.log 2>&1 || exit 1
for w in 1 2; do
  MAUV_SPLIT_W8=$w timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 5 --fused > gpurun_out/w82_cbf_$w.log 2>&1 || exit 1
done
MAUV_SPLIT_W8=2 timeout -k 10 600 $T tests/test_model_gpu.py > gpurun_out/w82_model.log 2>&1 || exit 1
MAUV_SPLIT_W8=2 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --steps 5 --warmup 1 > gpurun_out/w82_bench.log 2>&1 || exit 1
echo done
