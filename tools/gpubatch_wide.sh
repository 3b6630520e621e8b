# 128 x 256 16-bit tiles: parity, per-mode A/B (MAUV_P16_WIDE bitmask), bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py > gpurun_out/w_tests.log 2>&1 || { tail -30 gpurun_out/w_tests.log; exit 1; }
MAUV_P16_WIDE=7 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py > gpurun_out/w_tests7.log 2>&1 || { tail -30 gpurun_out/w_tests7.log; exit 1; }
tail -1 gpurun_out/w_tests.log gpurun_out/w_tests7.log
for W in 0 7; do
MAUV_P16_WIDE=$W timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --top 200 --trunks bathy --fused > gpurun_out/w_bf16_$W.log 2>&1 || exit 1
MAUV_P16_WIDE=$W timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --top 200 --trunks bathy --fused --only fwd --B 256 --G 2 > gpurun_out/w_inf_$W.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/w_bench.log 2>&1 || exit 1
tail -1 gpurun_out/w_bench.log
echo done
