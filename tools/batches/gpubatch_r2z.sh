# RECORD ONLY: the switch MAUV_P16_SHORT_DGRAD and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# short-K kernels: parity; bench A/B of the data-gradient variants and of the threshold
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels16_gpu.py tests/test_model16_gpu.py tests/test_dropin_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r2z_tests.log 2>&1 || { tail -30 gpurun_out/r2z_tests.log; exit 1; }
tail -1 gpurun_out/r2z_tests.log
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer-fp32"
for V in "1 256" "0 256" "1 256" "0 256" "1 512"; do
  set -- $V
  MAUV_P16_SHORT_DGRAD=$1 MAUV_P16_SHORT_K=$2 timeout -k 10 300 python -u $A > gpurun_out/r2z_b$1_$2.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r2z_b$1_$2.log').read().strip().splitlines()[-1]);print('dgrad$1 K$2', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
