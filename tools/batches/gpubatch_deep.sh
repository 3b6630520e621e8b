# RECORD ONLY: the switch MAUV_SPLIT_DEEP and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# A/B: three register stages (loads three tiles ahead) in the eight-wave 128x128 split kernel
# (record of a measured experiment whose code was removed: see DESIGN.md; the variable it sets is no longer read)
set -o pipefail
mkdir -p gpurun_out
MAUV_SPLIT_DEEP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_f32_math_gpu.py tests/test_model_gpu.py > gpurun_out/deep_tests.log 2>&1 || { tail -30 gpurun_out/deep_tests.log; exit 1; }
tail -n 1 gpurun_out/deep_tests.log
for P in 0 1; do
MAUV_SPLIT_DEEP=$P timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --top 3 --trunks bathy > gpurun_out/deep_cb_$P.log 2>&1 || exit 1
echo "P=$P $(grep 'TOTAL' gpurun_out/deep_cb_$P.log | tr '\n' ' ')"
done
for P in 0 1 0 1; do
MAUV_SPLIT_DEEP=$P timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 > gpurun_out/deep_b_$P.log 2>&1 || exit 1
echo "P=$P $(tail -n 1 gpurun_out/deep_b_$P.log | cut -c90-150)"
done
echo done
