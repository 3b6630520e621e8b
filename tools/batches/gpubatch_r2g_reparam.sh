# round 2g: reparam_sample with the MC groups split along blockIdx.y: sampling tests, an
# inference / training A/B against the previous library (libmauv_prev.so), then the full GPU
# suite and smoke() on the new library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py -m gpu -q -k "reparam or philox or sample" --timeout 120 --timeout-method thread > gpurun_out/r_tests.log 2>&1 || { tail -30 gpurun_out/r_tests.log; exit 1; }
tail -1 gpurun_out/r_tests.log
for L in prev hip prev hip; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer-fp32 --no-sweep > gpurun_out/r_b_$L.log 2>&1 || { tail -20 gpurun_out/r_b_$L.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r_b_$L.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2g_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r2g_tests.log | head; tail -5 gpurun_out/r2g_tests.log; exit 1; }
tail -1 gpurun_out/r2g_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2g_smoke.log 2>&1 || { tail -20 gpurun_out/r2g_smoke.log; exit 1; }
tail -1 gpurun_out/r2g_smoke.log
