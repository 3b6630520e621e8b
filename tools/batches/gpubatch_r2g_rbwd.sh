# round 2g: reparam_bwd with 64 input channels per block on the large 3x3 layers: reparam tests,
# then rocprofv3 kernel statistics of a serial bf16 step and a serial fp32 step with the previous
# library (libmauv_prev.so) and this one, and the bench training A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_model_gpu.py -m gpu -q -k "reparam or philox or train" --timeout 120 --timeout-method thread > gpurun_out/rb_tests.log 2>&1 || { tail -30 gpurun_out/rb_tests.log; exit 1; }
tail -1 gpurun_out/rb_tests.log
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 --no-sweep"
for L in prev hip; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_st16_$L -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C > gpurun_out/rb_st16_$L.log 2>&1 || exit 1
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_st32_$L -o run -- python3 bench.py --steps 2 --warmup 1 $C > gpurun_out/rb_st32_$L.log 2>&1 || exit 1
python3 -c "
import csv
for d in ('rb_st16_$L','rb_st32_$L'):
    r=list(csv.DictReader(open('gpurun_out/'+d+'/run_kernel_stats.csv')))
    x=[x for x in r if 'reparam_bwd' in x['Name']][0]
    print(d, x['Calls'], round(float(x['TotalDurationNs'])/3e6,3), 'ms/step', round(float(x['AverageNs'])/1e3,1), 'us avg')
"
done
for L in prev hip prev hip; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-sweep > gpurun_out/rb_b_$L.log 2>&1 || { tail -20 gpurun_out/rb_b_$L.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/rb_b_$L.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['bf16_train']['value'])"
done
