# 16-bit: skip the all-zero tile of an odd stage count; parity + per-shape + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py tests/test_model16_gpu.py > gpurun_out/o_tests.log 2>&1 || { tail -30 gpurun_out/o_tests.log; exit 1; }
tail -n 1 gpurun_out/o_tests.log
timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --top 200 --trunks bathy --fused > gpurun_out/o_bf16.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --top 200 --trunks bathy --fused --only fwd --B 256 --G 2 > gpurun_out/o_inf.log 2>&1 || exit 1
grep TOTAL gpurun_out/o_bf16.log gpurun_out/o_inf.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/o_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/o_bench.log | cut -c1-200
python3 -c "import json;d=json.loads(open('gpurun_out/o_bench.log').read().strip().splitlines()[-1]);print(d['inference']['value'], d['bf16_train']['value'])"
echo done
