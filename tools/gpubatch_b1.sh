set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/b1_model.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --steps 5 --warmup 1 > gpurun_out/b1_bench.log 2>&1 || exit 1
echo done
