# bench A/B: short-K forward kernels up to K = 256 vs the two-stage kernel only
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A="bench.py --steps 4 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer-fp32"
for K in 256 0 256 0 64; do
  MAUV_P16_SHORT_K=$K timeout -k 10 300 python -u $A > gpurun_out/r2y_b$K.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r2y_b$K.log').read().strip().splitlines()[-1]);print('K$K', d['value'], d['bf16_train']['value'], d['inference']['value'])"
done
