set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py tests/test_kernels16_gpu.py > gpurun_out/bs_kern.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/bs_model.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --no-cpu-baseline --exact-steps 0 > gpurun_out/bs_bench.log 2>&1 || exit 1
echo done
