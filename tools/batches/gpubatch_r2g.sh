# RECORD ONLY: the switch MAUV_LAZY_BN_INFER and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# A/B: inference with bn1/bn2 applied on load (default) vs materialised (MAUV_LAZY_BN_INFER=0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-bf16 --exact-steps 0 --no-roofline --no-infer-fp32"
timeout -k 10 300 python -u $A > gpurun_out/r2g_lazy.log 2>&1 || exit 1
MAUV_LAZY_BN_INFER=0 timeout -k 10 300 python -u $A > gpurun_out/r2g_mat.log 2>&1 || exit 1
timeout -k 10 300 python -u $A > gpurun_out/r2g_lazy2.log 2>&1 || exit 1
MAUV_LAZY_BN_INFER=0 timeout -k 10 300 python -u $A > gpurun_out/r2g_mat2.log 2>&1 || exit 1
for f in lazy mat lazy2 mat2; do python3 -c "import json;d=json.loads(open('gpurun_out/r2g_$f.log').read().strip().splitlines()[-1]);print('$f', d['inference']['value'], d['inference']['ms_per_batch'])"; done
