# 16-bit stems on the pipelined kernel: parity + stem timings + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py tests/test_model16_gpu.py > gpurun_out/s_tests.log 2>&1 || { tail -30 gpurun_out/s_tests.log; exit 1; }
tail -n 1 gpurun_out/s_tests.log
timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --top 6 --trunks bathy,sss --only fwd --B 256 --G 2 > gpurun_out/s_inf.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/s_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/s_bench.log
echo done
