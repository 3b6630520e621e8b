# short-K: fp32 split SEQ variant (MAUV_SPLIT_SHORT_K) parity + A/B; 16-bit sequential kernel
# for every K (MAUV_P16_SHORT_K=100000) per-layer
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_f32_math_gpu.py tests/test_model_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -1 gpurun_out/r3a_tests.log
for K in 256 0 256 0; do
  MAUV_SPLIT_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --only fwd --fused --top 200 > gpurun_out/r3a_f32_$K.log 2>&1 || exit 1
  echo split K$K $(grep "TOTAL fwd" gpurun_out/r3a_f32_$K.log)
done
for K in 100000 256; do
  MAUV_P16_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --G 20 --B 256 --only fwd --fused --top 200 > gpurun_out/r3a_f16_$K.log 2>&1 || exit 1
  echo p16 K$K $(grep "TOTAL fwd" gpurun_out/r3a_f16_$K.log)
done
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-bf16"
for K in 256 0 256 0; do
  MAUV_SPLIT_SHORT_K=$K timeout -k 10 300 python -u $A > gpurun_out/r3a_b$K.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3a_b$K.log').read().strip().splitlines()[-1]);print('split K$K', d['value'], d['inference']['value'], d['inference']['fp32']['value'])"
done
