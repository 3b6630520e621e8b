# round-2 evidence, part C: the default bench line after the MC chunk budget change, with the
# GPU tests that exercise the inference path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_dropin_gpu.py tests/test_model16_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2final_c_tests.log 2>&1 || { tail -20 gpurun_out/r2final_c_tests.log; exit 1; }
tail -1 gpurun_out/r2final_c_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/round2c_bench.log 2>&1 || { tail -20 gpurun_out/round2c_bench.log; exit 1; }
tail -1 gpurun_out/round2c_bench.log > gpurun_out/round2c_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/round2c_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], d['inference']['mc_chunk'], d['inference']['fp32']['value'], d['inference']['fp32']['mc_chunk'])"
