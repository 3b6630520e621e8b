# A/B: bn_bwd_partial with four rows in flight per thread (libmauv_hip.so) vs before (libmauv_bnold.so)
# (record of a measured experiment whose code was removed: see DESIGN.md; the variable it sets is no longer read)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels16_gpu.py -k "bn" > gpurun_out/bu_tests.log 2>&1 || { tail -30 gpurun_out/bu_tests.log; exit 1; }
tail -n 1 gpurun_out/bu_tests.log
for L in bnold hip bnold hip; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/bu_$L.log 2>&1 || exit 1
python3 -c "import json,sys;d=json.loads(open('gpurun_out/bu_$L.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['bf16_train']['value'])"
done
echo done
