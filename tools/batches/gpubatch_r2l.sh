# stems as one GEMM over shared im2col rows (MAUV_STEM_GEMM=1, default) vs per-sample implicit GEMMs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r2l_tests.log 2>&1 || { tail -30 gpurun_out/r2l_tests.log; exit 1; }
tail -1 gpurun_out/r2l_tests.log
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline"
for i in 1 2; do
timeout -k 10 300 python -u $A > gpurun_out/r2l_gemm$i.log 2>&1 || exit 1
MAUV_STEM_GEMM=0 timeout -k 10 300 python -u $A > gpurun_out/r2l_base$i.log 2>&1 || exit 1
done
for f in base1 gemm1 base2 gemm2; do python3 -c "import json;d=json.loads(open('gpurun_out/r2l_$f.log').read().strip().splitlines()[-1]);print('$f', d['value'], d['bf16_train']['value'], d['inference']['value'], d['inference'].get('fp32',{}).get('value'))"; done
