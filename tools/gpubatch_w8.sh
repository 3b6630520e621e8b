# eight-wave 128x128 split blocks: parity + timing vs four-wave
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
MAUV_SPLIT_W8=1 timeout -k 10 400 $T tests/test_f32_math_gpu.py tests/test_kernels_gpu.py > gpurun_out/w8_kern.log 2>&1 || exit 1
for w in 0 1; do
  MAUV_SPLIT_W8=$w timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 5 --fused > gpurun_out/w8_cbf_$w.log 2>&1 || exit 1
  MAUV_SPLIT_W8=$w MAUV_F32_MATH=split1 timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 5 --fused > gpurun_out/w8_cbf1_$w.log 2>&1 || exit 1
done
echo done
