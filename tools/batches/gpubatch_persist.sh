# RECORD ONLY: the switch MAUV_P16_PERSIST and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# A/B: persistent 16-bit conv blocks for short-K launches (MAUV_P16_PERSIST = max stages)
# (record of a measured experiment whose code was removed: see DESIGN.md; the variable it sets is no longer read)
set -o pipefail
mkdir -p gpurun_out
MAUV_P16_PERSIST=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels16_gpu.py tests/test_model16_gpu.py > gpurun_out/ps_tests.log 2>&1 || { tail -30 gpurun_out/ps_tests.log; exit 1; }
tail -n 1 gpurun_out/ps_tests.log
for P in 0 2 4 9; do
MAUV_P16_PERSIST=$P timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --top 200 --trunks bathy --fused --only fwd --B 256 --G 2 > gpurun_out/ps_inf_$P.log 2>&1 || exit 1
MAUV_P16_PERSIST=$P timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --top 200 --trunks bathy --fused > gpurun_out/ps_bf16_$P.log 2>&1 || exit 1
echo "P=$P inf $(grep 'TOTAL all' gpurun_out/ps_inf_$P.log) | bf16 $(grep 'TOTAL' gpurun_out/ps_bf16_$P.log | tr '\n' ' ')"
done
echo done
