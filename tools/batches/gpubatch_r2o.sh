# reparam kernels: wider reparam_bwd blocks, 32-bit sampling indices
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r2o_tests.log 2>&1 || { tail -30 gpurun_out/r2o_tests.log; exit 1; }
tail -1 gpurun_out/r2o_tests.log
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer"
timeout -k 10 300 python -u $A > gpurun_out/r2o_b1.log 2>&1 || exit 1
timeout -k 10 300 python -u $A > gpurun_out/r2o_b2.log 2>&1 || exit 1
for f in b1 b2; do python3 -c "import json;d=json.loads(open('gpurun_out/r2o_$f.log').read().strip().splitlines()[-1]);print('$f', d['value'], d['bf16_train']['value'])"; done
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2o_prof -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 > gpurun_out/r2o_prof.log 2>&1 || exit 1
f=$(ls gpurun_out/r2o_prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/r2o_prof -name "*kernel_stats.csv" | head -1)
grep -E "reparam|Name" "$f" | cut -c1-60,180-260
