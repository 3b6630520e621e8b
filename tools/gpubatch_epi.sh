# single-pass 16-bit epilogue: parity + per-shape + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py tests/test_model16_gpu.py > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -n 1 gpurun_out/e_tests.log
MAUV_P16_WIDE=0 timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --top 200 --trunks bathy --fused > gpurun_out/e_bf16.log 2>&1 || exit 1
MAUV_P16_WIDE=0 timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --top 200 --trunks bathy --fused --only fwd --B 256 --G 2 > gpurun_out/e_inf.log 2>&1 || exit 1
MAUV_P16_WIDE=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/e_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/e_bench.log
echo done
