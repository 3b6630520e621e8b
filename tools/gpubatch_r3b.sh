# the sequential one-buffer kernels for every forward K (16-bit: MAUV_P16_SHORT_K, fp32:
# MAUV_SPLIT_SHORT_K) vs K <= 256: bench A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline"
for K in 100000 256 100000 256; do
  MAUV_P16_SHORT_K=$K MAUV_SPLIT_SHORT_K=$K timeout -k 10 400 python -u $A > gpurun_out/r3b_b$K.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3b_b$K.log').read().strip().splitlines()[-1]);print('K$K', d['value'], d['bf16_train']['value'], d['inference']['value'], d['inference']['fp32']['value'])"
done
for K in 100000 256; do
  MAUV_SPLIT_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --only fwd --fused --top 200 > gpurun_out/r3b_f32_$K.log 2>&1 || exit 1
  MAUV_P16_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --only fwd --fused --top 200 > gpurun_out/r3b_b16_$K.log 2>&1 || exit 1
  echo K$K $(grep "TOTAL fwd" gpurun_out/r3b_f32_$K.log) / $(grep "TOTAL fwd" gpurun_out/r3b_b16_$K.log)
done
