set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 240 --timeout-method thread -k "two_channel" > gpurun_out/r2n_m.log 2>&1 || { tail -20 gpurun_out/r2n_m.log; exit 1; }
tail -2 gpurun_out/r2n_m.log
