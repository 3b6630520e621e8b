# round 2g: branch-free max-pool taps + XCD-contiguous order: pool tests, then the pool timing
# and the inference bench leg A/B against the previous library (libmauv_prev.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py -m gpu -q -k "pool" --timeout 120 --timeout-method thread > gpurun_out/p_tests.log 2>&1 || { tail -30 gpurun_out/p_tests.log; exit 1; }
tail -1 gpurun_out/p_tests.log
for L in prev hip prev hip; do
echo "== $L"
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 120 python -u tools/pool_bench.py || exit 1
done
for L in prev hip; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 300 python -u tools/infer_chunk.py 50 50 > gpurun_out/p_inf_$L.log 2>&1 || { tail -20 gpurun_out/p_inf_$L.log; exit 1; }
echo "$L: $(grep chunk gpurun_out/p_inf_$L.log | tr '\n' ' ')"
done
