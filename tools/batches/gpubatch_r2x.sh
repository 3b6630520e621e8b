# short-K 16-bit forward: one-stage (K = 64) and sequential one-buffer (K <= MAUV_P16_SHORT_K)
# variants vs the two-stage kernel (MAUV_P16_SHORT_K=0): parity, per-layer forward times, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MAUV_P16_SHORT_K=256 timeout -k 10 400 python -u -m pytest tests/test_kernels16_gpu.py tests/test_model16_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r2x_tests.log 2>&1 || { tail -30 gpurun_out/r2x_tests.log; exit 1; }
tail -1 gpurun_out/r2x_tests.log
for K in 64 128 256 0; do
  MAUV_P16_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --G 20 --B 256 --only fwd --fused --top 200 > gpurun_out/r2x_f16_$K.log 2>&1 || exit 1
  MAUV_P16_SHORT_K=$K timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --only fwd --fused --top 200 > gpurun_out/r2x_b16_$K.log 2>&1 || exit 1
  echo K$K $(grep "TOTAL fwd" gpurun_out/r2x_f16_$K.log) / $(grep "TOTAL fwd" gpurun_out/r2x_b16_$K.log)
done
