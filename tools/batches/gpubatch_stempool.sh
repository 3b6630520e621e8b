# fused stem bn1+ReLU+max-pool (MAUV_FUSED_STEM_POOL) and apply rows-per-thread 2/4: parity + A/B bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -n 1 gpurun_out/sp_tests.log
for cfg in "0 4" "1 4" "1 2" "0 4" "1 4" "1 2"; do
set -- $cfg
MAUV_FUSED_STEM_POOL=$1 MAUV_BN_APPLY_RPT=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/sp_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/sp_b.log').read().strip().splitlines()[-1]);print('fused=$1 rpt=$2', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
echo done
